set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/ka
for v in 0 1; do
  echo "== HIP_FORCE_DEV_KERNARG=$v"
  HIP_FORCE_DEV_KERNARG=$v timeout -k 5 60 ./tools/micro/rowchain_phase 25600 | head -4 || exit 1
  HIP_FORCE_DEV_KERNARG=$v timeout -k 5 60 ./tools/micro/attn_bwd_phase | sed -n 4,6p || exit 1
done
for v in 0 1 0 1; do
  HIP_FORCE_DEV_KERNARG=$v timeout -k 10 300 python bench.py --cpu-baseline-seconds 0 --steps 100 --warmup 20 > gpurun_out/ka/b$v.log 2>&1 || exit 1
  echo "kernarg dev=$v $(tail -1 gpurun_out/ka/b$v.log | cut -c90-140)"
done
