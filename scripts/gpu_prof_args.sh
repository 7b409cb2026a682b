#!/bin/bash
# kernel-trace profiles of the served bench under different bench.py argument sets:
#   ARMS="--h2d-wait host|--h2d-wait device" MODEL=deepfm   (arms separated by |, run in order, twice)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
case ${MODEL:-deepfm} in deepfm|wdl|dcn) sk="gemm_gather --min-us 80";; dlrm) sk="bottom_mlp3 --min-us 14";; *) sk="embed_pipe --min-us 30";; esac
IFS='|' read -ra arms <<< "$ARMS"
for rep in 1 2; do
  for i in "${!arms[@]}"; do
    d=gpurun_out/profarg_${i}_$rep
    rm -rf $d
    timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $d -o run --output-format rocpd \
      -- python3 bench.py --model ${MODEL:-deepfm} --steps 100 --warmup 10 --qps 0 ${arms[$i]} > $d.log 2>&1 \
      || { echo "prof arm $i failed"; tail -30 $d.log; exit 1; }
    db=$(find $d -name '*.db' | head -1)
    echo "== arm [${arms[$i]}] rep $rep: $(python -m tools.prof_summary "$db" --step-kernel $sk --from-kernel gemm | tail -1)"
  done
done
