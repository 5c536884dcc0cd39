// Sanitizer harness of the host-only code (the reference builds ASAN/UBSAN
// variants, cmake/Sanitizers.cmake:18-): the C ABI's parsers of untrusted bytes
// (3fs_amd/csrc/host_codec.cc) and the CPU oracle (oracle/crc_oracle.c), compiled with
// -fsanitize=address,undefined by tests/test_sanitizers.py and fed truncated, oversize and
// random inputs.  Any sanitizer report aborts (-fno-sanitize-recover); the harness also
// checks round trips and return codes, and prints one summary line.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "../../include/hf3fs_crc.h"
extern "C" {
#include "../../oracle/crc_oracle.h"
}

static int g_fail = 0;
#define CHECK(c)                                                       \
  do {                                                                 \
    if (!(c)) {                                                        \
      std::fprintf(stderr, "%s:%d CHECK(%s) failed\n", __FILE__, __LINE__, #c); \
      ++g_fail;                                                        \
    }                                                                  \
  } while (0)

// Heap copy of exactly n bytes, so that ASAN sees every read past the end.
static std::vector<uint8_t>* exact(const uint8_t* p, size_t n) { return new std::vector<uint8_t>(p, p + n); }

static void fuzz_checksum_serde(std::mt19937_64& rng, uint64_t& cases) {
  for (int t = 0; t < 3; ++t)
    for (uint32_t v : {0u, 1u, 0xFFEEAABBu, 0xFFFFFFFFu}) {  // TestSerdeObjectReader.cc:40,89,116
      uint8_t out[6];
      CHECK(hf3fs_checksum_serialize((uint8_t)t, v, out) == 6);
      for (uint64_t n = 0; n <= 6; ++n) {  // every truncation
        auto* b = exact(out, n);
        uint8_t ty = 9;
        uint32_t val = 7;
        uint64_t used = 0;
        const int rc = hf3fs_checksum_deserialize(b->data(), n, &ty, &val, &used);
        if (n == 6) CHECK(rc == 0 && ty == t && val == v && used == 6);
        else CHECK(rc == HF3FS_CRC_SERDE_INSUFFICIENT_LENGTH);
        delete b;
        ++cases;
      }
    }
  for (int it = 0; it < 200000; ++it) {  // random strings, varints included
    const size_t n = rng() % 24;
    std::vector<uint8_t> tmp(n);
    for (auto& x : tmp) x = (uint8_t)rng();
    if (n && rng() % 4 == 0) tmp[0] = (uint8_t)(rng() % 8);  // plausible lengths
    auto* b = exact(tmp.data(), n);
    uint8_t ty;
    uint32_t val;
    uint64_t used = 0;
    if (hf3fs_checksum_deserialize(n ? b->data() : nullptr, n, &ty, &val, &used) == 0) CHECK(used <= n);
    delete b;
    ++cases;
  }
  const uint8_t long_varint[12] = {0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0x01};
  uint8_t ty;
  uint32_t val;
  CHECK(hf3fs_checksum_deserialize(long_varint, sizeof(long_varint), &ty, &val, nullptr) != 0);
  CHECK(hf3fs_checksum_deserialize(nullptr, 4, &ty, &val, nullptr) == HF3FS_CRC_INVALID_ARG);
}

static std::vector<uint8_t> frames_of(std::mt19937_64& rng, int k) {
  std::vector<uint8_t> b;
  for (int i = 0; i < k; ++i) {
    const uint32_t sz = rng() % 3 == 0 ? 0 : (uint32_t)(rng() % 300);
    const uint32_t ck = 0x86u | (uint32_t)(rng() & 1) | (uint32_t)(rng() << 8);
    for (int j = 0; j < 4; ++j) b.push_back((uint8_t)(ck >> (8 * j)));
    for (int j = 0; j < 4; ++j) b.push_back((uint8_t)(sz >> (8 * j)));
    for (uint32_t j = 0; j < sz; ++j) b.push_back((uint8_t)rng());
  }
  return b;
}

static void fuzz_frame_walk(std::mt19937_64& rng, uint64_t& cases) {
  std::vector<hf3fs_crc_frame> fr(512);
  for (int it = 0; it < 300; ++it) {
    const int k = 1 + (int)(rng() % 40);
    const std::vector<uint8_t> good = frames_of(rng, k);
    uint64_t nf = 0, used = 0;
    {
      auto* b = exact(good.data(), good.size());
      CHECK(hf3fs_crc_frame_walk(b->data(), good.size(), fr.data(), fr.size(), &nf, &used) == 0);
      CHECK(nf == (uint64_t)k && used == good.size());
      for (uint64_t i = 0; i < nf; ++i) CHECK(fr[i].offset + fr[i].size <= good.size());
      delete b;
    }
    for (size_t cut = 0; cut < good.size(); cut += 1 + rng() % 7) {  // truncations
      auto* b = exact(good.data(), cut);
      const int rc = hf3fs_crc_frame_walk(cut ? b->data() : nullptr, cut, fr.data(), fr.size(), &nf, &used);
      CHECK(used <= cut);
      if (rc == 0) CHECK(used == cut);
      delete b;
      ++cases;
    }
    std::vector<uint8_t> bad = good;  // oversize length fields, non-serde headers
    const size_t at = (rng() % k) ? 0 : 0;
    const uint32_t huge = 0xFFFFFFF0u + (uint32_t)(rng() % 16);
    std::memcpy(&bad[at + 4], &huge, 4);
    {
      auto* b = exact(bad.data(), bad.size());
      CHECK(hf3fs_crc_frame_walk(b->data(), bad.size(), fr.data(), fr.size(), &nf, &used) == HF3FS_CRC_INVALID_ARG);
      delete b;
    }
    bad = good;
    bad[0] = 0x11;
    {
      auto* b = exact(bad.data(), bad.size());
      CHECK(hf3fs_crc_frame_walk(b->data(), bad.size(), fr.data(), fr.size(), &nf, &used) == HF3FS_CRC_INVALID_ARG);
      delete b;
    }
    {  // max_frames smaller than the stream: stops without overrunning the output
      const uint64_t cap = rng() % (k + 1);
      std::vector<hf3fs_crc_frame>* out = new std::vector<hf3fs_crc_frame>(cap);
      auto* b = exact(good.data(), good.size());
      CHECK(hf3fs_crc_frame_walk(b->data(), good.size(), cap ? out->data() : nullptr, cap, &nf, &used) == 0);
      CHECK(nf == cap);
      delete b;
      delete out;
    }
    cases += 4;
  }
  for (int it = 0; it < 100000; ++it) {  // random bytes
    const size_t n = rng() % 64;
    std::vector<uint8_t> tmp(n);
    for (auto& x : tmp) x = (uint8_t)rng();
    if (n >= 1 && rng() % 2) tmp[0] = (uint8_t)(0x86 | (rng() & 1));
    auto* b = exact(tmp.data(), n);
    uint64_t nf = 0, used = 0;
    (void)hf3fs_crc_frame_walk(n ? b->data() : nullptr, n, fr.data(), fr.size(), &nf, &used);
    CHECK(used <= n);
    delete b;
    ++cases;
  }
}

static void fuzz_engine_meta(std::mt19937_64& rng, uint64_t& cases) {
  for (int it = 0; it < 20000; ++it) {
    hf3fs_crc_engine_meta m{};
    m.pos = rng();
    m.chain_ver = (uint32_t)rng();
    m.chunk_ver = (uint32_t)rng();
    m.len = (uint32_t)rng();
    m.checksum = (uint32_t)rng();
    m.timestamp = rng();
    m.last_request_id = rng();
    m.last_client_low = rng();
    m.last_client_high = rng();
    m.etag_len = (uint8_t)(rng() % (sizeof(m.etag) + 1));
    for (uint32_t j = 0; j < m.etag_len; ++j) m.etag[j] = (char)rng();
    m.uncommitted = (uint8_t)(rng() & 1);
    uint8_t buf[256];
    uint64_t w = 0;
    CHECK(hf3fs_crc_engine_meta_encode(&m, buf, sizeof(buf), &w) == 0);
    for (uint64_t n = 0; n <= w; n += (n + 8 < w ? 1 + rng() % 8 : 1)) {  // truncations
      auto* b = exact(buf, n);
      hf3fs_crc_engine_meta back{};
      uint64_t used = 0;
      const int rc = hf3fs_crc_engine_meta_decode(n ? b->data() : buf, n, &back, &used);
      if (n == w) {
        CHECK(rc == 0 && used == w && back.checksum == m.checksum && back.pos == m.pos &&
              back.etag_len == m.etag_len && !std::memcmp(back.etag, m.etag, m.etag_len) &&
              back.uncommitted == m.uncommitted);
      } else {
        CHECK(rc == HF3FS_CRC_INVALID_ARG);
      }
      delete b;
      ++cases;
    }
    uint8_t small[8];
    CHECK(hf3fs_crc_engine_meta_encode(&m, small, rng() % 8, &w) == HF3FS_CRC_INVALID_ARG);
    hf3fs_crc_engine_meta bad = m;
    bad.etag_len = (uint8_t)(sizeof(m.etag) + 1 + rng() % 100);
    CHECK(hf3fs_crc_engine_meta_encode(&bad, buf, sizeof(buf), &w) == HF3FS_CRC_INVALID_ARG);
  }
  for (int it = 0; it < 100000; ++it) {  // random bytes, plausible body lengths
    const size_t n = rng() % 140;
    std::vector<uint8_t> tmp(n);
    for (auto& x : tmp) x = (uint8_t)rng();
    if (n && rng() % 2) tmp[0] = (uint8_t)(rng() % 128);
    if (n > 58 && rng() % 2) tmp[57] = (uint8_t)(rng() % 40);
    auto* b = exact(tmp.data(), n);
    hf3fs_crc_engine_meta back{};
    uint64_t used = 0;
    if (hf3fs_crc_engine_meta_decode(n ? b->data() : tmp.data(), n, &back, &used) == 0) CHECK(used <= n);
    delete b;
    ++cases;
  }
  char et[8];
  for (uint32_t v : {0u, 1u, 0xFu, 0x10u, 0xDEADBEEFu, 0xFFFFFFFFu}) {
    const uint32_t k = hf3fs_crc_default_etag(v, et);
    CHECK(k >= 1 && k <= 8);
  }
}

static void fuzz_algebra(std::mt19937_64& rng, uint64_t& cases) {
  for (int it = 0; it < 50000; ++it) {
    uint8_t ty = (uint8_t)(rng() % 5);  // 3, 4: unknown types
    uint32_t v = (uint32_t)rng();
    const uint8_t ot = (uint8_t)(rng() % 5);
    const int rc = hf3fs_checksum_combine(&ty, &v, ot, (uint32_t)rng(), rng() % 3 ? rng() : 0);
    CHECK(rc == 0 || rc == HF3FS_CRC_CHECKSUM_MISMATCH || rc == HF3FS_CRC_INVALID_ARG);
    (void)hf3fs_crc_shift((uint8_t)(rng() % 4), (uint32_t)rng(), rng());
    ++cases;
  }
  CHECK(hf3fs_checksum_combine(nullptr, nullptr, 1, 0, 1) == HF3FS_CRC_INVALID_ARG);
}

static void fuzz_oracle(std::mt19937_64& rng, uint64_t& cases) {
  std::vector<uint8_t> pool(1 << 16);
  for (auto& x : pool) x = (uint8_t)rng();
  for (int it = 0; it < 3000; ++it) {  // every kernel of the CRC restatement on exact-size buffers
    const size_t n = rng() % 700;
    auto* b = exact(pool.data() + rng() % 1000, n);
    const uint8_t* p = n ? b->data() : nullptr;
    const uint32_t s = (uint32_t)rng();
    const uint32_t hw = orc_crc32c_hw(s, p, n), sw = orc_crc32c_sw(s, p, n);
    CHECK(hw == sw && sw == orc_crc_bitwise(s, p, n, 0x82F63B78u));
    CHECK(orc_crc32_sw(s, p, n) == orc_crc_bitwise(s, p, n, 0xEDB88320u));
    const size_t cut = n ? rng() % n : 0;
    CHECK(orc_crc32c_combine(orc_crc32c_hw(s, p, cut), orc_crc32c_hw(0, p ? p + cut : nullptr, n - cut), n - cut) ==
          hw);
    delete b;
    ++cases;
  }
  for (int it = 0; it < 3000; ++it) {  // ChunkReplica::updateChecksum and the engine write on random IOs
    const uint32_t cap = 1 + (uint32_t)(rng() % 9000);
    std::vector<uint8_t>* chunk = new std::vector<uint8_t>(cap);
    for (auto& x : *chunk) x = (uint8_t)rng();
    const uint32_t size_after = (uint32_t)(rng() % (cap + 1));
    const uint32_t off = (uint32_t)(rng() % (cap + 1)), len = off < cap ? (uint32_t)(rng() % (cap - off + 1)) : 0;
    orc_checksum out{}, cck{(uint8_t)(rng() % 3), (uint32_t)rng()}, wck{(uint8_t)(rng() % 3), (uint32_t)rng()};
    int kase = -1;
    const int rc = orc_replica_update_checksum_case(chunk->data(), size_after, cck, wck, off, len, (int)(rng() & 1),
                                                    (uint32_t)(rng() % (cap + 1)), (int)(rng() & 1), &out, &kase);
    CHECK(rc != 0 || (kase >= 1 && kase <= 4));
    uint32_t elen = (uint32_t)(rng() % (cap + 1)), eck = (uint32_t)rng();
    const uint32_t dlen = off < cap ? (uint32_t)(rng() % (cap - off + 1)) : 0;
    std::vector<uint8_t>* data = new std::vector<uint8_t>(dlen);
    for (auto& x : *data) x = (uint8_t)rng();
    const uint32_t dck = orc_rs_crc32c(dlen ? data->data() : nullptr, dlen);
    const int erc = orc_engine_write_case(chunk->data(), &elen, &eck, cap, dlen ? data->data() : nullptr, dlen, off,
                                          dck, (int)(rng() % 4 == 0), 0, (int)(rng() % 8 != 0), &kase);
    CHECK(erc != 0 || (kase >= 1 && kase <= 4 && elen <= cap));
    delete data;
    delete chunk;
    ++cases;
  }
}

int main() {
  std::mt19937_64 rng(0x5A417E);
  uint64_t cases = 0;
  fuzz_checksum_serde(rng, cases);
  fuzz_frame_walk(rng, cases);
  fuzz_engine_meta(rng, cases);
  fuzz_algebra(rng, cases);
  fuzz_oracle(rng, cases);
  std::printf("{\"fuzz_host_codec\":\"%s\",\"cases\":%llu,\"failures\":%d}\n", g_fail ? "FAILED" : "ok",
              (unsigned long long)cases, g_fail);
  return g_fail ? 1 : 0;
}
