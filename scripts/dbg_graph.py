"""Debug: verify_blocks captured in a hipGraph, variants (queue / static)."""
import importlib, os, sys
import numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
hf = importlib.import_module("3fs_amd"); L = hf._lib; L.load()
dev = torch.device("cuda:0")
rng = np.random.default_rng(44)
size = 96 << 20
arena = torch.randint(0, 256, (size,), dtype=torch.uint8, device=dev)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 30000
lens = rng.choice([4096, 8192, 16384, 32768, 65536], n).astype(np.uint32)
offs = (rng.integers(0, (size - 65536) // 4096, n) * 4096).astype(np.uint64)
O = torch.tensor(offs.view(np.int64), device=dev); Ls = torch.tensor(lens.view(np.int32), device=dev)
E = torch.zeros(n, dtype=torch.int32, device=dev)
mism = torch.zeros(n, dtype=torch.uint8, device=dev); cnt = torch.zeros(1, dtype=torch.int32, device=dev)
comp = torch.zeros(n, dtype=torch.int32, device=dev)
cs = torch.cuda.Stream(dev)
with torch.cuda.stream(cs):
    L.verify_blocks(1, arena, O, Ls, E, mism, cnt, n, 65536, computed=comp, stream=cs)
cs.synchronize()
want = comp.clone()
E.copy_(want)
with torch.cuda.stream(cs):
    L.verify_blocks(1, arena, O, Ls, E, mism, cnt, n, 65536, computed=comp, stream=cs)
cs.synchronize()
print("eager: cnt", int(cnt.item()), "equal", bool(torch.equal(comp, want)))
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g, stream=cs):
    L.verify_blocks(1, arena, O, Ls, E, mism, cnt, n, 65536, computed=comp, stream=cs)
for r in range(3):
    comp.zero_(); cnt.fill_(-1); mism.fill_(7); torch.cuda.synchronize()
    g.replay(); torch.cuda.synchronize()
    print("replay", r, "cnt", int(cnt.item()), "comp==want", bool(torch.equal(comp, want)),
          "nz comp", int((comp != 0).sum().item()), "mism sum", int(mism.sum().item()))
