# round 4: C3 decode-attention knobs (variant, beam rows per XCD group) at 4 batches in flight
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4_c3attn
mkdir -p $O
S="beam_xcd=5,decode_attn5=6;beam_xcd=1,decode_attn5=6;beam_xcd=10,decode_attn5=6;beam_xcd=5,decode_attn5=5;beam_xcd=5,decode_attn5=4;beam_xcd=5,decode_attn5=3;beam_xcd=5,decode_attn5=2;beam_xcd=5,decode_attn5=6"
timeout -k 10 600 python -u tools/c3_probe.py 4 1024 "$S" > $O/probe.txt 2>&1 || { tail -30 $O/probe.txt; exit 1; }
cat $O/probe.txt
