set -o pipefail
D=apex_dqn_amd/ops/_build/libapex_kernels_debug.so
for v in base NOEPI NOPERM BOTH; do
  cp exp_libs/dbg_$v.so $D || exit 1
  echo "== $v" >> gpurun_out/exp.log
  timeout -k 10 100 python -u scripts/probe_conv12.py --probe >> gpurun_out/exp.log 2>&1 || exit 1
done
