#!/bin/bash
# Counter passes (rocprofv3 --pmc, one run per pass, each under its own KILL
# timeout) over the serving-shape forwards of DeepFM (16384 rows) and DCN-v2
# fp8 (8192 rows), plus the hipBLASLt comparison at the same GEMM shapes.
# Slot budget per pass (MI355X): <= 8 SQ, <= 4 TCC (FETCH_SIZE = 3, WRITE_SIZE = 2), <= 2 GRBM.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/ctr
rm -rf $OUT && mkdir -p $OUT
timeout -s KILL 60 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
PASS_SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
PASS_FETCH="FETCH_SIZE GRBM_GUI_ACTIVE"
PASS_WRITE="WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"
for model in deepfm dcn_v2; do
  rows=16384; [ $model = dcn_v2 ] && rows=8192
  i=0
  for pass in "$PASS_SQ" "$PASS_FETCH" "$PASS_WRITE"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $pass --kernel-trace --output-format csv -d $OUT/${model}_p$i -o run \
      -- python3 -m distributed_tf_serving_amd.bench.kernel_drive --model $model --rows $rows --iters 10 \
      > $OUT/${model}_p$i.log 2>&1 || { echo "pass $i of $model failed"; tail -5 $OUT/${model}_p$i.log; exit 1; }
  done
  python -m distributed_tf_serving_amd.bench.counters_summary $OUT --title "counters" > /dev/null
done
for model in deepfm dcn_v2; do
  mkdir -p $OUT/sum_$model && cp -r $OUT/${model}_p* $OUT/sum_$model/ 2>/dev/null
  python -m distributed_tf_serving_amd.bench.counters_summary $OUT/sum_$model \
    --title "$model serving-shape forward, 1 MI355X (rocprofv3 --pmc, 3 passes)" > $OUT/summary_$model.md
  cat $OUT/summary_$model.md
done
timeout -k 10 300 python -u -m distributed_tf_serving_amd.bench.microbench --serving > $OUT/microbench.jsonl 2>&1 \
  || { echo "microbench failed"; tail -5 $OUT/microbench.jsonl; exit 1; }
cat $OUT/microbench.jsonl | grep '^{'
