#!/bin/bash
# A/B of two library builds on the vocabulary GEMM probe, alternating in one GPU session:
#   A = librecsys_hip.$A.so (RS_LIB_VARIANT), B = the in-tree library.  PROBE_ARGS passed through.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for i in $(seq ${ROUNDS:-2}); do
  for v in A B; do
    if [ $v = A ]; then e="RS_LIB_VARIANT=${A:-a}"; else e="RS_AB_B=1"; fi
    env $e timeout -k 10 200 python tools/diag/vocab_gemm_probe.py --only n256 $PROBE_ARGS 2>&1 | sed "s/^/$v /" | grep n256 || exit 1
  done
done
