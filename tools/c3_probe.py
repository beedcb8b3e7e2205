#!/usr/bin/env python3
"""C3 (beam 5, eval batches of 256) throughput at several in-flight depths (bench.py c3_beam5),
optionally under zs_tune_set knob sets (";"-separated "k=v,k=v", each reset to 0 after):
    python tools/c3_probe.py [inflight=2,4] [clips=1024] [sets]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "zero-shot-aac_amd"))
import torch  # noqa: E402

import bench  # noqa: E402

os.environ["GPU_MAX_HW_QUEUES"] = "16"


def main():
    infl = [int(c) for c in (sys.argv[1] if len(sys.argv) > 1 else "2,4").split(",")]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    sets = (sys.argv[3] if len(sys.argv) > 3 else "").split(";")
    from zsaac._lib import call
    args = bench.parse([])
    dev = torch.device("cuda", 0)
    for k in infl:
        for ks in sets:
            kv = dict(x.split("=") for x in ks.split(",") if x)
            for key, v in kv.items():
                call("zs_tune_set", key.encode(), int(v))
            r = bench.c3_beam5(args, dev, n, k)
            for key in kv:
                call("zs_tune_set", key.encode(), 0)
            print(json.dumps({"inflight": k, "clips": n, "knobs": ks, "value": r["value"]}),
                  flush=True)


if __name__ == "__main__":
    main()
