#!/usr/bin/env python3
"""Where the workgroups of k concurrent persistent decode grids land (HW_ID / XCC_ID read by each
workgroup, zs_decode_persist_set_stamps step -2): how many CUs host 0 / 1 / 2 / .. grid workgroups,
and how many CUs host workgroups of two different grids.

    python tools/placement.py [grid=96] [k=2,3,5]
"""
import collections
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "zero-shot-aac_amd"))
import torch  # noqa: E402

import bench  # noqa: E402

os.environ["GPU_MAX_HW_QUEUES"] = "16"
WS_X = 4096 + 3 * 64 * 768 * 2 + 64 * 3072 * 2      # decode_grid.hip's workspace layout


def main():
    G = int(sys.argv[1]) if len(sys.argv) > 1 else 96
    ks = [int(k) for k in (sys.argv[2] if len(sys.argv) > 2 else "2,3,5").split(",")]
    from zsaac import ops
    from zsaac._lib import call

    class A:
        batch, dtype, encoder, mapper, beam, entry_length, group, compact = \
            64, "bf16", "htsat", "mlp", 0, 67, 1, 1
        encoder_batch = 64
    dev = torch.device("cuda", 0)
    pipe, _, _ = bench.build(A, dev)
    wav = bench.synthetic_clips(64, 0, dev)
    kmax = max(ks)
    pipes = [pipe] + [pipe.twin() for _ in range(kmax - 1)]
    streams = ops.dedicated_streams(kmax, dev)
    for p, s in zip(pipes, streams):
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            p.caption_wav(wav)
        p.decoder.persist_grid = G
    torch.cuda.synchronize()
    call("zs_decode_persist_set_stamps", None, -2, None)
    for k in ks:
        for p, s in zip(pipes[:k], streams[:k]):
            with torch.cuda.stream(s):
                p.decoder.greedy_begin(64)
        torch.cuda.synchronize()
        where = []
        for p in pipes[:k]:
            ws = p.decoder.persist_ws
            v = ws[WS_X:WS_X + 8 * G].view(torch.int64).cpu().tolist()
            where.append([((x >> 32) & 0xff, (x >> 8) & 0xff) for x in v])   # XCC, SE|SH|CU
        per_cu = collections.Counter(c for g in where for c in g)
        grids_per_cu = collections.Counter()
        for c in per_cu:
            grids_per_cu[sum(1 for g in where if c in g)] += 1
        print(json.dumps({"grid": G, "k": k, "cus_used": len(per_cu),
                          "wgs_per_cu_hist": dict(collections.Counter(per_cu.values())),
                          "grids_per_cu_hist": dict(grids_per_cu),
                          "xcd_of_wg0_first8": [where[0][w][0] for w in range(8)]}), flush=True)
    call("zs_decode_persist_set_stamps", None, 0, None)


if __name__ == "__main__":
    main()
