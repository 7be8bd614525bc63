# fp32 step rate vs the split-K reduction rows of the conv3 / conv2 weight gradients
# (SW.wg_rows3 / SW.wg_rows2 through APEX_SWITCHES; 0 = ops/conv.py default).
# Usage (through gpurun): bash scripts/wg_rows_sweep.sh TAG "384 704" "256 704" ...
TAG=$1; shift
args=()
for v in "$@"; do set -- $v; args+=("APEX_SWITCHES=wg_rows3=$1,wg_rows2=$2 :: --no-bf16-extra"); done
AB_STEPS=400 AB_WARMUP=40 bash scripts/gpu.sh ab "$TAG" "${args[@]}"
