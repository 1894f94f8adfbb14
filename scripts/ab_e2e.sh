# A/B of the per-frame drop-in loop (harness/e2e_bench) against abvar/base/libcrlot_dsp.so
# (LD_LIBRARY_PATH beats the harness's RUNPATH), alternating processes.
set -u
mkdir -p gpurun_out
for i in 1 2 3; do
  for lib in new base; do
    for nh in "256 200 1024" "256 200 960"; do
      if [ $lib = base ]; then pre="env LD_LIBRARY_PATH=$PWD/abvar/base"; else pre=""; fi
      out=$(timeout -k 10 60 $pre harness/e2e_bench $nh | tail -1) || exit 1
      echo "{\"lib\": \"$lib\", \"args\": \"$nh\", \"r\": $out}"
    done
  done
done
