set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/ab2
cd $R
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 tools/membench.hip -o tools/membench && \
timeout -k 10 300 python -m pytest tests -m gpu -q -x > gpurun_out/ab2/pytest.log 2>&1 && \
timeout -k 10 200 ./tools/membench 32 > gpurun_out/ab2/membench.json 2>&1 && \
timeout -k 10 500 python tools/kbench.py --rounds 5 > gpurun_out/ab2/kbench.json 2> gpurun_out/ab2/kbench.err
echo rc=$?
tail -3 gpurun_out/ab2/pytest.log
