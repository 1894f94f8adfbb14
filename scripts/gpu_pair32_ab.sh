# Half-wave K_pair walker (CRLOT_PAIR32=1, pair32.hip) vs K_pair at the headline
# (needs a library built with -DCRLOT_PAIR32_EXPERIMENT: make -C crlot-dsp_amd/csrc with pair32.o rebuilt under that flag)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
CRLOT_PAIR32=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "roundtrip_vs_oracle or golden_e2e or full_scale" > gpurun_out/p32_tests.log 2>&1; echo "pair32 tests rc=$? $(tail -1 gpurun_out/p32_tests.log)"
: > gpurun_out/p32_ab.jsonl
for rep in 1 2 3; do
  for cfg in "base:" "p32c6:CRLOT_PAIR32=1" "p32c4:CRLOT_PAIR32=1 CRLOT_CHUNKS=4" "p32c8:CRLOT_PAIR32=1 CRLOT_CHUNKS=8" "basec8:CRLOT_CHUNKS=8"; do
    name=${cfg%%:*}; envs=${cfg#*:}
    v=$(env $envs timeout -k 10 120 python bench.py --no-strong --no-cpu-baseline --steps 50 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.readline()); print(d['value'], d['roofline']['kernel_ms'])") || exit 1
    echo "{\"cfg\": \"$name\", \"rep\": $rep, \"value_kernel_ms\": \"$v\"}" >> gpurun_out/p32_ab.jsonl
  done
done
cat gpurun_out/p32_ab.jsonl
