import importlib, sys, time, torch
sys.path.insert(0, '.')
sfm = importlib.import_module('3d_reconstruction_amd')
abi = importlib.import_module('3d_reconstruction_amd._abi')
dev = torch.device('cuda', 0)
g = torch.Generator(device=dev); g.manual_seed(7)
nr = 1 << 20
o = torch.rand((nr, 3), generator=g, device=dev) * 64 - 32
d = torch.randn((nr, 3), generator=g, device=dev)
far = torch.rand((nr, 1), generator=g, device=dev) * 64
rays = torch.cat([o, d / d.norm(dim=1, keepdim=True), torch.zeros_like(far), far], 1).contiguous()
for rep in range(3):
    steps = torch.empty(nr, dtype=torch.int32, device=dev)
    torch.cuda.synchronize(); t0 = time.perf_counter()
    abi.call("sfmhip_voxel_traversal_count", rays.data_ptr(), nr, 1.0, 1 << 20, steps.data_ptr(), abi.stream_ptr())
    torch.cuda.synchronize(); t1 = time.perf_counter()
    S = 1 + int(steps.max().item()); t2 = time.perf_counter()
    out = torch.empty((nr, S, 3), dtype=torch.float32, device=dev); torch.cuda.synchronize(); t3 = time.perf_counter()
    abi.call("sfmhip_voxel_traversal", rays.data_ptr(), nr, 1.0, S, out.data_ptr(), abi.stream_ptr())
    torch.cuda.synchronize(); t4 = time.perf_counter()
    print(f"S={S} count {1e3*(t1-t0):.2f} ms, max {1e3*(t2-t1):.2f}, alloc {1e3*(t3-t2):.2f}, fill {1e3*(t4-t3):.2f} ms; mean steps {steps.float().mean().item():.1f}; out {out.numel()*4/1e9:.2f} GB")
