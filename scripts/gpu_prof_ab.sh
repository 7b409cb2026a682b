#!/bin/bash
# kernel-trace profile of the served bench under each value of an env toggle: AB_VAR=X AB_VALUES="0 1" MODEL=dlrm
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
case ${MODEL:-deepfm} in deepfm|wdl|dcn) sk="gemm_gather --min-us 80";; dlrm) sk="bottom_mlp3 --min-us 14";; *) sk="embed_pipe --min-us 30";; esac
for v in $AB_VALUES; do
  d=gpurun_out/profab_${MODEL}_$v
  rm -rf $d
  env $AB_VAR=$v timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $d -o run --output-format rocpd \
    -- python3 bench.py --model ${MODEL:-deepfm} --steps 100 --warmup 10 --qps 0 > $d.log 2>&1 \
    || { echo "prof $v failed"; tail -30 $d.log; exit 1; }
  db=$(find $d -name '*.db' | head -1)
  python -m tools.prof_summary "$db" --steps 1100 --step-kernel $sk --from-kernel "${FROM:-gemm}" \
    --title "bench.py live path (${MODEL}, $AB_VAR=$v), 1 MI355X" > gpurun_out/profab_${MODEL}_$v.md
  echo "== $AB_VAR=$v"; head -16 gpurun_out/profab_${MODEL}_$v.md | tail -12; tail -1 gpurun_out/profab_${MODEL}_$v.md
done
