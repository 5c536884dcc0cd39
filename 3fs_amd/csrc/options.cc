// options.cc -- the process's tuning / test switches (options.h) and their C ABI
// (hf3fs_crc_set_option / hf3fs_crc_get_option, include/hf3fs_crc.h).
#include "options.h"

#include <cctype>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>

#include "../../include/hf3fs_crc.h"
#include "internal.h"

namespace hf3fs_crc {
namespace {

// A switch: its name (HF3FS_CRC_<NAME upper-cased> in the environment), the
// accepted range, and for enumerations the value names (index - 1 = stored value).
struct Spec {
  const char* name;
  std::atomic<int>* i;
  std::atomic<uint32_t>* u;
  int64_t lo, hi;
  const char* names[3];  // enumerations: values -1, 0, 1 spelled out (also accepted: the numbers)
  bool test_only = false;  // set only through hf3fs_crc_set_option, never from the environment
};

Options g_opts;

const Spec* specs(size_t* n) {
  Options& o = g_opts;
  static const Spec s[] = {
      {"nt", &o.nt, nullptr, 0, 1, {}},
      {"seg_kib", nullptr, &o.seg_kib, 0, 1 << 20, {}},
      {"static", &o.static_stride, nullptr, 0, 1, {}},
      {"pipe", &o.pipe, nullptr, -1, 1, {"auto", "0", "1"}},
      {"balance", &o.balance, nullptr, 0, 1, {}},
      {"record_direct", &o.record_direct, nullptr, 0, 1, {}},
      {"update_pipeline", &o.update_pipeline, nullptr, -1, 1, {"mode", "unfused", "fused"}},
      {"apply_pieces", nullptr, &o.apply_pieces, 1, 64, {}},
      {"apply_min_kib", nullptr, &o.apply_min_kib, 1, 1 << 20, {}},
      {"apply_nt", nullptr, &o.apply_nt, 0, 7, {}},
      {"apply_grid", &o.apply_grid, nullptr, -1, 2, {}},
      {"apply_piece_kib", nullptr, &o.apply_piece_kib, 4, 16, {}},
      {"prehash_rep", nullptr, &o.prehash_rep, 1, 8, {}},
      {"frame_stream", &o.frame_stream, nullptr, -1, 1, {"auto", "0", "1"}},
      {"frame_segw", nullptr, &o.frame_segw, 1, 64, {}},
      {"debug", &o.debug, nullptr, 0, 1, {}},
      {"poison", nullptr, &o.poison, 0, 0xFFFFFFFFll, {}, true},
      {"audit", &o.audit, nullptr, 0, 1, {}},
      {"range_stream", &o.range_stream, nullptr, 0, 1, {}},
      {"list_runs", &o.list_runs, nullptr, 0, 1, {}},
      {"fault_io", nullptr, &o.fault_io, 0, 0xFFFFFFFFll, {}, true},
  };
  *n = sizeof(s) / sizeof(s[0]);
  return s;
}

const Spec* find(const char* name) {
  size_t n = 0;
  const Spec* s = specs(&n);
  for (size_t k = 0; k < n; ++k)
    if (!strcmp(s[k].name, name)) return &s[k];
  return nullptr;
}

// value text -> stored value; false if it is not one of the switch's values
bool parse(const Spec& sp, const char* text, int64_t* out) {
  if (!text || !*text) return false;
  if (sp.names[0])
    for (int k = 0; k < 3; ++k)
      if (!strcmp(text, sp.names[k])) {
        *out = k - 1;
        return true;
      }
  char* end = nullptr;
  const long long v = strtoll(text, &end, 0);
  if (*end || v < sp.lo || v > sp.hi) return false;
  *out = v;
  return true;
}

void store(const Spec& sp, int64_t v) {
  if (sp.i)
    sp.i->store((int)v);
  else
    sp.u->store((uint32_t)v);
}

int64_t value_of(const Spec& sp) { return sp.i ? (int64_t)sp.i->load() : (int64_t)sp.u->load(); }

// Switches of earlier rounds: still set in someone's environment, never read again.
const char* const kRetired[] = {"HF3FS_CRC_UPDATE_UNFUSED", "HF3FS_CRC_APPLY_SHFL", "HF3FS_CRC_APPLY_ALIGN",
                                "HF3FS_CRC_NO_POOL",        "HF3FS_CRC_SYNC_FREE",  "HF3FS_CRC_DELTA_PIECE_KIB",
                                "HF3FS_CRC_DELTA_LAG"};

void snapshot_environment() {
  size_t n = 0;
  const Spec* s = specs(&n);
  for (size_t k = 0; k < n; ++k) {
    std::string env = "HF3FS_CRC_";
    for (const char* c = s[k].name; *c; ++c) env += (char)toupper((unsigned char)*c);
    const char* text = getenv(env.c_str());
    if (!text) continue;
    if (s[k].test_only) {  // fault injection never comes from a production environment
      fprintf(stderr, "[hf3fs_crc] ignoring %s: a test-only switch, settable only through hf3fs_crc_set_option\n",
              env.c_str());
      continue;
    }
    int64_t v = 0;
    if (parse(s[k], text, &v))
      store(s[k], v);
    else
      fprintf(stderr, "[hf3fs_crc] ignoring %s=%s (not a value of this switch; the default stays)\n", env.c_str(),
              text);
  }
  for (const char* r : kRetired)
    if (getenv(r)) fprintf(stderr, "[hf3fs_crc] %s is no longer read (DESIGN.md 4.0)\n", r);
}

std::once_flag g_once;

}  // namespace

Options& options() {
  std::call_once(g_once, snapshot_environment);
  return g_opts;
}

}  // namespace hf3fs_crc

using namespace hf3fs_crc;

extern "C" {

int hf3fs_crc_set_option(const char* name, const char* value) {
  options();  // the environment snapshot first, so it never overwrites a later override
  if (!name) return fail(HF3FS_CRC_INVALID_ARG, "null option name");
  const Spec* sp = find(name);
  if (!sp) return fail(HF3FS_CRC_INVALID_ARG, "unknown option '%s'", name);
  int64_t v = 0;
  if (!parse(*sp, value, &v)) return fail(HF3FS_CRC_INVALID_ARG, "option '%s': bad value '%s'", name, value ? value : "");
  store(*sp, v);
  return HF3FS_CRC_OK;
}

int hf3fs_crc_get_option(const char* name, char* out, size_t cap) {
  options();
  if (!name || !out || cap == 0) return fail(HF3FS_CRC_INVALID_ARG, "null argument");
  const Spec* sp = find(name);
  if (!sp) return fail(HF3FS_CRC_INVALID_ARG, "unknown option '%s'", name);
  const int64_t v = value_of(*sp);
  if (sp->names[0])
    snprintf(out, cap, "%s", sp->names[v + 1]);
  else
    snprintf(out, cap, "%lld", (long long)v);
  return HF3FS_CRC_OK;
}

}  // extern "C"
