set -o pipefail
mkdir -p gpurun_out
for k in 128 256 576 1024 2048; do
  timeout -k 10 120 python -u -m tools.studies.microbench --variants "16384,1024,$k:14,18" >> gpurun_out/kscan.log 2>&1 || { tail -20 gpurun_out/kscan.log; exit 1; }
done
grep '^{' gpurun_out/kscan.log | python -c "
import sys, json
for l in sys.stdin:
    d=json.loads(l); print(d['K'], 'v14', d['v14_us'], 'v18', d['v18_us'], 'lib', d['hipblaslt_us'])"
