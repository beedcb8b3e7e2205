import ctypes, os, sys, torch
lib = ctypes.CDLL(os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "tools/hip/libcuhog.so"))
lib.xcc_probe.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
for n in (24, 64, 192, 512):
    out = torch.full((n,), -1, dtype=torch.int32, device="cuda")
    lib.xcc_probe(n, out.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    v = out.cpu().tolist()
    ok = sum(1 for i, x in enumerate(v) if (x & 0xf) == i % 8)
    print(n, "matches blockIdx%8:", ok, "/", n, "first 24:", v[:24])
