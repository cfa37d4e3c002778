set -o pipefail
out=gpurun_out/qa_ab2.txt
: > $out
for cfg in f1 f0 f1b f0b f1c f0c; do
  v=0; [[ $cfg == f1* ]] && v=1
  POLYKEY_QKV_ATTN_FUSED=$v timeout -k 10 240 python tools/ab_decode.py --steps 128 --reps 3 --tag $cfg >> $out 2> gpurun_out/qa_ab.err || exit 1
done
cat $out
CONC=64 bash tools/gpu/r3_prof.sh
