set -o pipefail
for r in 1 2 3; do echo "== new $r" >> gpurun_out/dbg2.log; timeout -k 10 60 python -u scripts/experiments/dbg_wq.py >> gpurun_out/dbg2.log 2>&1 || exit 1; done
for r in 1 2 3; do echo "== head $r" >> gpurun_out/dbg2.log; APEX_BUILD_DIR=$PWD/exp_build timeout -k 10 60 python -u scripts/experiments/dbg_wq.py >> gpurun_out/dbg2.log 2>&1 || exit 1; done
