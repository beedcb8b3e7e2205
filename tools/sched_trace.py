"""Host-side schedule trace of the bench's staged headline: per timed repetition, when each
begin group was enqueued and each batch's grid launched / seen done (ms from the run's start),
with the repetition's wall time.  argv: clips (1280) reps (6).  One JSON line per repetition."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
clips = int(sys.argv[1]) if len(sys.argv) > 1 else 1280
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 6
os.environ["ZSAAC_RUNNER_TRACE"] = "1"
sys.argv = ["bench.py", "--no-cpu-baseline"]
import bench  # noqa: E402
import torch  # noqa: E402

args = bench.parse()
dev = torch.device("cuda", 0)
pipe, _, _ = bench.build(args, dev)
dt, outs, runner, info = bench.run_captions(args, 1, 0, dev, pipe, clips, 0, [clips], args.inflight,
                                            5, reps=reps)
traces = getattr(runner, "traces", [])[-reps:]
for t_s, tr in zip(info["timed_reps_s"], traces):
    ev = {}
    for kind, i, ms in tr:
        ev.setdefault(kind, {})[i] = ms
    print(json.dumps({"rep_s": t_s, "begin_group_ms": ev.get("begin_group"),
                      "launch_ms": ev.get("launch"), "done_ms": ev.get("done")}), flush=True)
