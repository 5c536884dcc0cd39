import sys, os, ctypes, importlib
sys.path.insert(0, '.'); sys.path.insert(0, 'oracle')
import numpy as np, torch, oracle as orc
hf = importlib.import_module("3fs_amd"); L = hf._lib
dev = torch.device("cuda:0")
rng = np.random.default_rng(7)
host = rng.integers(0, 256, 8 << 20, dtype=np.uint8)
d = torch.from_numpy(host).to(dev)
off, ln = 5670495, 8189
want = orc.crc32c_raw(host[off:off+ln])
print("want", want)
for n_extra, max_len in [(0, 8189), (0, 70000), (0, 3 << 20), (1, 70000), (1, 3<<20), (5, 3<<20)]:
    addrs = [d.data_ptr() + off] + [d.data_ptr() + 100 * (i+1) for i in range(n_extra)]
    lens = [ln] + [min(max_len, 65536 + 1000 * i) for i in range(n_extra)]
    n = len(addrs)
    A = torch.tensor(np.array(addrs, dtype=np.uint64).view(np.int64), device=dev)
    Ln = torch.tensor(lens, dtype=torch.int64, device=dev)
    out = torch.zeros(n, dtype=torch.int32, device=dev)
    L.create_batch(1, A, Ln, out, n, max_len)
    torch.cuda.synchronize()
    got = int(out[0].item()) & 0xFFFFFFFF
    print("dev-desc", n_extra, max_len, got, got == want)
# coalescer single request
with L.Coalescer(device=0) as co:
    v = co.create_one(1, d.data_ptr() + off, ln)
    print("coal", v, v == want)
    for m in [1, 2, 15, 16, 17, 4096]:
        o2 = off - (off % 16) + (m % 16) + 32
        for l2 in [8189, 100, 1000, 1023, 1024, 1025, 4096, 65536, 65537]:
            v = co.create_one(1, d.data_ptr() + o2, l2)
            w = orc.crc32c_raw(host[o2:o2+l2])
            if v != w: print("coal mismatch", o2 % 16, l2)
