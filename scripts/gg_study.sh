timeout -k 10 200 python -u -m tools.studies.microbench --gather-gemm > gpurun_out/gg_study.log 2>&1 || { tail -20 gpurun_out/gg_study.log; exit 1; }
grep '^{' gpurun_out/gg_study.log
