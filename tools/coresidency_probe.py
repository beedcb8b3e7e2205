#!/usr/bin/env python3
"""How fast does a bs-64 begin (encode + prompt + mapper + prefill + step 0) run beside resident
"grids" that hold their CUs the way the persistent decode does (tools/hip/cu_hog.hip: resident,
asleep, WAVES x 256 VGPRs + LDS each), full-CU hogs vs half-CU ones -- the case for a persistent
decode that leaves room on its CUs.

    python tools/coresidency_probe.py [reps=5]
"""
import ctypes
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "zero-shot-aac_amd"))
import torch  # noqa: E402

import bench  # noqa: E402

os.environ["GPU_MAX_HW_QUEUES"] = "16"


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    from zsaac import ops
    hog = ctypes.CDLL(os.path.join(ROOT, "tools", "hip", "libcuhog.so"))
    hog.cu_hog_launch.argtypes = [ctypes.c_int] * 3 + [ctypes.c_void_p] * 3
    args = bench.parse([])
    dev = torch.device("cuda", 0)
    pipe, _, _ = bench.build(args, dev)
    pipe.decoder.persist = False          # begin work only (no decode launch at its end)
    wav = bench.synthetic_clips(64, 0, dev)
    main_s = ops.dedicated_streams(1, dev)[0]
    hog_s = ops.dedicated_streams(10, dev)
    with torch.cuda.stream(main_s):
        for _ in range(3):
            pipe.begin_wav(wav)
    torch.cuda.synchronize()
    res = {}
    for name, waves, lds, ngrids in (("none", 0, 0, 0), ("full8w_110k_x5", 8, 110 * 1024, 5),
                                     ("half4w_48k_x5", 4, 48 * 1024, 5),
                                     ("full8w_110k_x10", 8, 110 * 1024, 10),
                                     ("half4w_48k_x10", 4, 48 * 1024, 10),
                                     ("half4w_48k_x20", 4, 48 * 1024, 20),
                                     ("none", 0, 0, 0)):
        flag = torch.zeros(1, dtype=torch.int32, device=dev)
        out = torch.zeros(1, dtype=torch.int32, device=dev)
        torch.cuda.synchronize()
        try:
            if ngrids:      # one launch of 24 x ngrids workgroups (no queue-sharing question)
                rc = hog.cu_hog_launch(waves, 24 * ngrids, lds, flag.data_ptr(), out.data_ptr(),
                                       hog_s[0].cuda_stream)
                assert rc == 0, rc
            time.sleep(0.02)
            ts = []
            for _ in range(reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                with torch.cuda.stream(main_s):
                    e0.record()
                    pipe.begin_wav(wav)
                    e1.record()
                e1.synchronize()
                ts.append(e0.elapsed_time(e1))
        finally:
            with torch.cuda.stream(main_s):
                flag.fill_(1)
            torch.cuda.synchronize()
        print(json.dumps({"hogs": name, "begin_ms": round(statistics.median(ts), 3),
                          "hog_exit": int(out[0])}), flush=True)


if __name__ == "__main__":
    main()
