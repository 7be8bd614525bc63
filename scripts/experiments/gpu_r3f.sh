# Split IMPALA: band-variant tests, then a sweep of the row bands on the fp32 IMPALA bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_impala_split.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r3f.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_r3f.log; [ $rc -eq 0 ] || exit $rc
I="--network impala --no-bf16-extra"
AB_STEPS=200 AB_WARMUP=20 bash scripts/ab.sh isplit ":: $I" "APEX_ISPLIT_BANDS=rb16x42=10 :: $I" "APEX_ISPLIT_BANDS=rb16x42=7 :: $I" \
  "APEX_ISPLIT_BANDS=sc16x16x42p0=21 :: $I" "APEX_ISPLIT_BANDS=sc16x16x42p0=14 :: $I" \
  "APEX_ISPLIT_BANDS=sc32x16x42p0=11 :: $I" "APEX_ISPLIT_BANDS=sc16x32x42p1=6 :: $I" \
  "APEX_ISPLIT_BANDS=sc32x32x21p1=8 :: $I" "APEX_ISPLIT_BANDS=rb32x21=11 :: $I" "APEX_ISPLIT_BANDS=sc32x32x21p0=11 :: $I"
