cd $GRAFT_REPO_ROOT
echo "== off/off"; DBG_A=0 DBG_B=0 timeout -k 10 120 python scripts/dbg_fp32_c1f_model.py 2>&1 | grep -v amdgpu.ids | head -14
echo "== on/on"; DBG_A=1 DBG_B=1 timeout -k 10 120 python scripts/dbg_fp32_c1f_model.py 2>&1 | grep -v amdgpu.ids | head -14
