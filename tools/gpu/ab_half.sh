# decode-step A/B: fp32 split-K slabs from 128-row (default) vs 64-row n-blocks at half the split
set -o pipefail
out=gpurun_out/ab_half.txt
: > $out
for cfg in "base:" "o4:4096x4096:4" "down4:4096x14336:4" "both4:4096x4096:4,4096x14336:4" "base2:"; do
  tag=${cfg%%:*}; val=${cfg#*:}
  POLYKEY_SKINNY_HALF="$val" timeout -k 10 240 python tools/ab_decode.py --steps 128 --reps 3 --tag $tag >> $out 2> gpurun_out/ab_half.err || exit 1
done
