"""Does a caption run leave the process slower?  Times fixed single-stream workloads (encoder
pass, one bs-64 caption, a 1280 x 768 x 3072 GEMM) before and after bench.run_captions with the
given schedule (argv: begin_first 0|1, pipelines' batches), and after the runner is deleted.
Prints one JSON line (ms per workload at each point)."""
import gc
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
bf = sys.argv[1] if len(sys.argv) > 1 else "1"
nclips = int(sys.argv[2]) if len(sys.argv) > 2 else 1280
sys.argv = ["bench.py", "--begin-first", bf, "--no-cpu-baseline"]
import bench  # noqa: E402  (sets GPU_MAX_HW_QUEUES from argv before torch initialises HIP)
import torch  # noqa: E402
from zsaac import ops  # noqa: E402

args = bench.parse()
dev = torch.device("cuda", 0)
pipe, _, _ = bench.build(args, dev)
wav = bench.synthetic_clips(64, 0, dev)
a = torch.randn(1280, 3072, device=dev).to(torch.bfloat16)
w = torch.randn(768, 3072, device=dev).to(torch.bfloat16)
o = torch.empty(1280, 768, device=dev, dtype=torch.bfloat16)


def timeit(fn, n):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    e1.synchronize()
    return round(e0.elapsed_time(e1) / n, 4)


def probe():
    return {"encode64_ms": timeit(lambda: pipe.encode(wav), 10),
            "caption64_ms": timeit(lambda: pipe.caption_wav(wav), 3),
            "gemm_us": round(1e3 * timeit(lambda: ops.gemm(a, w, o), 200), 2)}


big = torch.empty(2**30, device=dev)
big.fill_(1.0)
res = {"begin_first": bf, "before": probe(), "stream4g_ms_before": timeit(lambda: big.sum(), 5)}
del big
dt, outs, runner, info = bench.run_captions(args, 1, 0, dev, pipe, nclips, 0, [nclips], args.inflight,
                                            5, reps=3)
res["run_s"] = info["timed_reps_s"]
res["pipes"] = len(runner.pipes)
res["after_run"] = probe()
del runner, outs
gc.collect()
torch.cuda.synchronize()
torch.cuda.empty_cache()
res["after_del"] = probe()
# a pipeline built after the run (fresh weights and buffers), and a fresh 4 GiB stream
pipe_a = pipe
pipe, _, _ = bench.build(args, dev)
res["new_pipe_after"] = probe()
pipe = pipe_a
big = torch.empty(2**30, device=dev)
big.fill_(1.0)
res["stream4g_ms_after"] = timeit(lambda: big.sum(), 5)
res["mem_alloc_gb"] = round(torch.cuda.memory_allocated() / 2**30, 2)
res["mem_reserved_gb"] = round(torch.cuda.memory_reserved() / 2**30, 2)
print(json.dumps(res))
