#!/bin/bash
# Round-5 pass AA: SQ counter passes over the dW and forward labs (where the
# row / K loops' cycles go: waits, issue stalls, LDS, matrix-core busy).
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
cd "$ROOT"
O=gpurun_out/r05aa
mkdir -p $O
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
P2="SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_FLAT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU GRBM_GUI_ACTIVE"
for b in dw_lab fwd_lab; do
  for p in 1 2; do
    eval C=\$P$p
    timeout -s KILL 120 rocprofv3 --pmc $C -d $O/${b}_p$p -o run --output-format csv -- tools/bin/$b > $O/${b}_p$p.log 2>&1 || { tail -5 $O/${b}_p$p.log; exit 1; }
    python3 tools/lab/pmc_lab.py $O/${b}_p$p | tee $O/${b}_p$p.txt | grep -v flush
  done
done
