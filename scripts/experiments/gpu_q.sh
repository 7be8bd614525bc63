set -o pipefail
rm -f gpurun_out/dbg2.log
for r in 1 2; do echo "== new $r" >> gpurun_out/dbg2.log; timeout -k 10 60 python -u scripts/experiments/dbg_wq.py >> gpurun_out/dbg2.log 2>&1 || exit 1; done
for r in 1 2; do echo "== head $r" >> gpurun_out/dbg2.log; APEX_BUILD_DIR=$PWD/exp_build timeout -k 10 60 python -u scripts/experiments/dbg_wq.py >> gpurun_out/dbg2.log 2>&1 || exit 1; done
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_split.py tests/test_gpu_conv.py tests/test_gpu_fc128.py > gpurun_out/t.log 2>&1
timeout -k 10 120 python -u scripts/probe_conv12.py > gpurun_out/p.log 2>&1 && timeout -k 10 120 python -u scripts/probe_conv12.py --probe >> gpurun_out/p.log 2>&1 && timeout -k 10 240 python -u scripts/bench_cu_steal.py > gpurun_out/steal.log 2>&1
