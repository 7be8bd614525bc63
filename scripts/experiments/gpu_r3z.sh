# Optimizer launch block-count sweep (APEX_OPT_BLOCKS) on the final tree, both precisions.
set -o pipefail
AB_STEPS=600 AB_WARMUP=50 bash scripts/ab.sh optblk "APEX_OPT_BLOCKS=512 :: --no-bf16-extra" "APEX_OPT_BLOCKS=384 :: --no-bf16-extra" \
  "APEX_OPT_BLOCKS=256 :: --no-bf16-extra" "APEX_OPT_BLOCKS=512 :: --dtype bf16 --no-bf16-extra" \
  "APEX_OPT_BLOCKS=384 :: --dtype bf16 --no-bf16-extra" "APEX_OPT_BLOCKS=256 :: --dtype bf16 --no-bf16-extra"
