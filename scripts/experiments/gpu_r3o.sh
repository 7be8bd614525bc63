# fc forward K-split sweep (192 blocks at 2 splits on 256 CUs).
set -o pipefail
AB_STEPS=600 AB_WARMUP=50 bash scripts/ab.sh fcks "APEX_FC_KSPLIT=2 :: --no-bf16-extra" "APEX_FC_KSPLIT=3 :: --no-bf16-extra" \
  "APEX_FC_KSPLIT=4 :: --no-bf16-extra" "APEX_FC_KSPLIT=5 :: --no-bf16-extra" \
  "APEX_FC_KSPLIT=2 :: --dtype bf16 --no-bf16-extra" "APEX_FC_KSPLIT=4 :: --dtype bf16 --no-bf16-extra" \
  "APEX_FC_KSPLIT=5 :: --dtype bf16 --no-bf16-extra"
