set -u
cd $GRAFT_REPO_ROOT
bash tools/gpu_exp.sh || exit $?
PMC_CMD="python3 $GRAFT_REPO_ROOT/tools/exp_dense.py --apply 4 --index 2 --layouts 0,1 --rounds 1 --steps 2" PMC_GROUPS="TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum;TCC_EA0_RDREQ_DRAM_sum;TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_DRAM_sum" bash tools/gpu_pmc.sh
