#!/usr/bin/env python3
"""The f32 parity mode (bench.py f32_parity_mode) at several clip counts / in-flight depths, and
zs_tune_set knob sets (each line's value under every set in turn):
    python tools/f32_probe.py [clips=384,1045] [inflight=10] [sets=";"-separated "k=v,k=v"]"""
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
    clips = [int(c) for c in (sys.argv[1] if len(sys.argv) > 1 else "384,1045").split(",")]
    infl = [int(c) for c in (sys.argv[2] if len(sys.argv) > 2 else "10").split(",")]
    sets = (sys.argv[3] if len(sys.argv) > 3 else "").split(";")
    from zsaac._lib import call
    args = bench.parse([])
    dev = torch.device("cuda", 0)
    for n in clips:
        for k in infl:
            for ks in sets:
                kv = dict(x.split("=") for x in ks.split(",") if x)
                for key, v in kv.items():
                    call("zs_tune_set", key.encode(), int(v))
                r = bench.sub_run(args, dev, torch.float32, 1, k, n, 1)
                for key in kv:                       # (the knobs used here default to 0)
                    call("zs_tune_set", key.encode(), 0)
                print(json.dumps({"clips": n, "inflight": k, "knobs": ks, "value": r["value"],
                                  "decode_steps_mean": r["config"].get("decode_steps_mean")}),
                      flush=True)


if __name__ == "__main__":
    main()
