set -e
for i in 1 2; do
for cfg in "CRLOT_GATHER=3" "CRLOT_GATHER=3 CRLOT_GATHER_BPB=1" "CRLOT_GATHER=3 CRLOT_GATHER_BPB=2" "CRLOT_GATHER=2"; do
  env $cfg timeout -k 10 200 python bench.py --suite ola > gpurun_out/o.json
  python3 -c "
import json,sys
d=json.loads(open('gpurun_out/o.json').read().strip().splitlines()[-1]); print(sys.argv[1], [(r['frame'],r['hop'],round(r['gpu_msamples_s']/1000)) for r in d['grid']])
" "$cfg"
done
done
