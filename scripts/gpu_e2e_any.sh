set -o pipefail
mkdir -p gpurun_out
for nh in "1024 256" "960 480" "882 441"; do
  set -- $nh
  timeout -k 10 120 ./harness/e2e_bench $2 200 $1 > gpurun_out/e2e_${1}_$2.json || { echo "e2e $1/$2 failed"; exit 1; }
  cat gpurun_out/e2e_${1}_$2.json
done
