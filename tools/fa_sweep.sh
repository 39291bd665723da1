cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for nt in 640 512 1024; do
 FMX_FA_NT=$nt timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k rank > gpurun_out/fa_t$nt.log 2>&1 || { tail -30 gpurun_out/fa_t$nt.log; exit 1; }
 echo "NT=$nt tests: $(tail -1 gpurun_out/fa_t$nt.log)"
 FMX_FA_NT=$nt timeout -k 10 120 python tools/kbench.py --ops cs_rank 2>&1 | grep -v amdgpu | head -1
done
