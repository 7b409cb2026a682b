set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/models
for m in dcn_v2 dlrm wdl dcn; do
  timeout -k 10 240 python -u bench.py --model $m --steps 200 --warmup 20 --qps 0 > gpurun_out/models/$m.log 2>&1 || { echo "$m failed"; tail -20 gpurun_out/models/$m.log; exit 1; }
  grep '^{"metric' gpurun_out/models/$m.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(sys.argv[1], round(d["value"]/1e6,2), d["ms_per_step"], d["config"]["global_batch"], d.get("p50_request_ms"), d["config"]["model"])' $m
done
