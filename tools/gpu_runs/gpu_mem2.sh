set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/mem2
cd $R
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 tools/membench.hip -o tools/membench && \
timeout -k 10 300 ./tools/membench 40 > gpurun_out/mem2/membench.json 2>&1
echo rc=$?
