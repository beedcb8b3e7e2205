#!/bin/bash
# the default Mistral C5 bench line
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r2mb}; mkdir -p $O
timeout -k 10 300 python bench.py --mistral > $O/mistral_bench.json 2> $O/m.err || { tail $O/m.err; exit 1; }
tail -1 $O/mistral_bench.json | cut -c1-200
