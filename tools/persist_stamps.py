#!/usr/bin/env python3
"""Phase timing inside the persistent decode (zs_decode_persist_set_stamps): per barrier of one
decode step, the median over workgroups of the compute before it (previous wait end -> arrive),
the wait (arrive -> wait end) and the arrival skew (last - first arrive), in microseconds.
bg > 0: the traced grid runs beside bg other batches' grids of the same size (pipeline twins on
their own streams, decode only), the load of the headline.

    python tools/persist_stamps.py [step=3] [grid=48] [bg=0] [dtype=bf16]

dtype f32: the f32 parity mode's grid decode (zs_gpt2_decode_persist_f32, grid 192).
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "zero-shot-aac_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    step = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    from zsaac import ops
    from zsaac._lib import call

    f32 = len(sys.argv) > 4 and sys.argv[4] == "f32"

    class A:
        batch, dtype, encoder, mapper, beam, entry_length, group, compact = \
            64, "f32" if f32 else "bf16", "htsat", "mlp", 0, 67, 1, 1
        encoder_batch = 64
    dev = torch.device("cuda", 0)
    pipe, _, _ = bench.build(A, dev, dtype=torch.float32 if f32 else torch.bfloat16)
    wav = bench.synthetic_clips(64, 0, dev)
    pipe.caption_wav(wav)
    G = 192 if f32 else ops.decode_persist_grid(int(sys.argv[2]) if len(sys.argv) > 2 else 48)
    nbg = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    pipes = [pipe] + [pipe.twin() for _ in range(nbg)]
    streams = ops.dedicated_streams(len(pipes), dev)
    for p, s in zip(pipes, streams):
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            p.caption_wav(wav)
        p.decoder.persist_grid = G
    torch.cuda.synchronize()
    buf = torch.zeros(G, 128, dtype=torch.int64, device=dev)
    dec = pipe.decoder
    call("zs_decode_persist_set_stamps", buf.data_ptr(), step, dec.persist_ws.data_ptr())
    for _ in range(3):
        for p, s in reversed(list(zip(pipes, streams))):   # the traced grid last
            with torch.cuda.stream(s):
                p.decoder.greedy_begin(64)
        torch.cuda.synchronize()
    call("zs_decode_persist_set_stamps", None, 0, None)
    t = buf.cpu().numpy().astype(np.float64) / 100.0     # us (100 MHz)
    if os.environ.get("STAMPS_OUT"):                      # raw stamps for offline analysis
        np.save(os.environ["STAMPS_OUT"], t)
    start, end = t[:, 127], t[:, 126]
    names = []
    for l in range(12):
        names += [f"L{l}.A qkv", f"L{l}.B attn", f"L{l}.C proj", f"L{l}.D fc", f"L{l}.E mproj"]
    names.append("F lmhead")
    t0 = np.median(start)
    prev = start.copy()
    rows, comp, wait = [], [], []
    for i, nm in enumerate(names):
        arr, wt = t[:, 2 * i], t[:, 2 * i + 1]
        c, w = arr - prev, wt - arr
        rows.append({"phase": nm, "compute_med": round(float(np.median(c)), 2),
                     "compute_max": round(float(np.max(c)), 2),
                     "wait_med": round(float(np.median(w)), 2),
                     "arrive_skew": round(float(arr.max() - arr.min()), 2),
                     "end_at": round(float(np.median(wt) - t0), 1)})
        comp.append(c)
        wait.append(w)
        prev = wt
    g_phase = end - prev
    for r in rows[:5] + rows[-6:]:
        print(json.dumps(r))
    kinds = {"A": [], "B": [], "C": [], "D": [], "E": []}
    for r in rows[:-1]:
        kinds[r["phase"].split(".")[1][0]].append((r["compute_med"], r["wait_med"], r["compute_max"]))
    summ = {k: {"compute_med": round(float(np.mean([a for a, _, _ in v])), 2),
                "compute_max": round(float(np.mean([c for _, _, c in v])), 2),
                "wait_med": round(float(np.mean([b for _, b, _ in v])), 2)} for k, v in kinds.items()}
    summ["F"] = {"compute_med": rows[-1]["compute_med"], "wait_med": rows[-1]["wait_med"]}
    summ["G"] = round(float(np.median(g_phase)), 2)
    summ["step_us"] = round(float(np.median(end - start)), 1)
    print(json.dumps({"grid": G, "background_grids": nbg, "per_phase_kind_mean_us": summ}))
    # phase F per workgroup, and by blockIdx % 8 (the XCD under round-robin dispatch)
    # does a workgroup that is slow in one phase stay slow in the next?  (rank correlation of
    # per-workgroup compute times of consecutive phases, and how often the last arrival of a
    # barrier is also among the slowest quarter of the next phase)
    cm = np.array(comp[:-1])
    rk = np.argsort(np.argsort(cm, axis=1), axis=1).astype(np.float64)
    cors = [float(np.corrcoef(rk[i], rk[i + 1])[0, 1]) for i in range(len(rk) - 1)]
    last_slow = [int(np.argmax(cm[i]) in set(np.argsort(-cm[i + 1])[:max(1, G // 4)]))
                 for i in range(len(cm) - 1)]
    print(json.dumps({"rank_corr_next_phase_mean": round(float(np.mean(cors)), 3),
                      "slowest_in_next_quarter_frac": round(float(np.mean(last_slow)), 3),
                      "compute_mean_over_phases": round(float(cm.mean()), 2),
                      "compute_max_over_phases": round(float(cm.max(axis=1).mean()), 2)}))
    fc = comp[-1]
    print(json.dumps({"F_compute_by_wg": [round(float(x), 1) for x in fc],
                      "F_compute_by_wg_mod8": [round(float(np.mean(fc[k::8])), 1) for k in range(8)],
                      "F_slowest_wg": [int(i) for i in np.argsort(-fc)[:6]]}))


if __name__ == "__main__":
    main()
