# A/B of vocabulary-GEMV launch variants (kernel time via wmi_bench_kernel 0)
set -o pipefail
export WMI_MODEL_CACHE=/tmp/wmi_models
for v in "WMI_LOGITS_G=1" "WMI_LOGITS_G=2" "WMI_LOGITS_G=2 WMI_LOGITS_CAP=768" "WMI_LOGITS_G=2 WMI_LOGITS_CAP=1024" "WMI_LOGITS_G=2 WMI_LOGITS_CAP=2048" "WMI_LOGITS_G=4 WMI_LOGITS_CAP=256" "WMI_LOGITS_G=4 WMI_LOGITS_CAP=512"; do
  echo -n "$v: "; timeout -k 10 120 env $v python scripts/kernel_probe.py base 0 50 || exit 1
done
