set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 --json-extra > gpurun_out/fresh_deepfm.log 2>&1 || { tail -20 gpurun_out/fresh_deepfm.log; exit 1; }
grep -E '^\{"metric|server_us_per_step' gpurun_out/fresh_deepfm.log | cut -c1-400
for v in "16384,1024,544:14,17,18" "16384,1024,1024:14,17,18" "16384,512,1024:10,14,17" "16384,512,64:4,10,14" "16384,256,512:4,10,14"; do
  timeout -k 10 120 python -u -m tools.studies.microbench --variants "$v" >> gpurun_out/dlrm_variants.log 2>&1 || { tail -20 gpurun_out/dlrm_variants.log; exit 1; }
done
cat gpurun_out/dlrm_variants.log | grep '^{'
