#!/usr/bin/env python3
"""The bench's f32 parity-mode line alone (1045 clips, bs 64, 10 batches in flight) -- run it under
rocprofv3 --kernel-trace --stats to see where the f32 mode's time goes.

    python tools/f32_profile.py [clips=1045] [inflight=10]
"""
import json
import os
import sys
from types import SimpleNamespace

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "zero-shot-aac_amd"))
import torch  # noqa: E402

import bench  # noqa: E402

os.environ["GPU_MAX_HW_QUEUES"] = "16"


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1045
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    args = SimpleNamespace(dtype="f32", group=1, encoder="htsat", mapper="mlp", batch=64,
                           encoder_batch=0, beam=0, entry_length=67, compact=1, persist_budget=0,
                           encode_ahead=256)
    res = bench.sub_run(args, torch.device("cuda", 0), torch.float32, 1, k, n, 1)
    print(json.dumps({"value": res["value"], "ms_per_step": res["ms_per_step"]}), flush=True)


if __name__ == "__main__":
    main()
