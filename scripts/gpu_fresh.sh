# fresh-box behaviour: the same bench 3x back to back (json-extra host stats) + GPU clocks between runs
set -o pipefail
mkdir -p gpurun_out/fresh
(timeout 20 rocm-smi --showclocks --showpower --showtemp > gpurun_out/fresh/smi_0.txt 2>&1 || true)
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 --json-extra > gpurun_out/fresh/run_$i.log 2>&1 || { tail -20 gpurun_out/fresh/run_$i.log; exit 1; }
  (timeout 20 rocm-smi --showclocks --showpower --showtemp > gpurun_out/fresh/smi_$i.txt 2>&1 || true)
  grep '^{"metric' gpurun_out/fresh/run_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('run $i', round(d['value']/1e6,2), 'M', d['ms_per_step'], d['server'])"
  grep server_us_per_step gpurun_out/fresh/run_$i.log | cut -c1-200
done
