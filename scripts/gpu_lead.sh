set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/lead
DTFS_TRACE=1 timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --memory-copy-trace -d gpurun_out/lead -o run --output-format rocpd \
  -- python3 bench.py --model ${MODEL:-deepfm} --steps 100 --warmup 10 --qps 0 > gpurun_out/lead.log 2>&1 || { tail -30 gpurun_out/lead.log; exit 1; }
db=$(find gpurun_out/lead -name '*.db' | head -1)
python -m tools.studies.launch_lead "$db" ${LEAD_ARGS:-}
