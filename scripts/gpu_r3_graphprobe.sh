# round 3: does hipGraphLaunch (and hipLaunchKernel) block the host on this ROCm?  The probe
# under the runtime's dispatch / graph knobs (each its own process)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/r3g
run() { echo "== $*"; env "$@" timeout -k 10 120 python -u benchmarks/graph_launch_probe.py >> gpurun_out/r3g/probe.log 2>&1 || { tail gpurun_out/r3g/probe.log; exit 1; }; tail -1 gpurun_out/r3g/probe.log; }
run LK_X=default
run DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
run DEBUG_CLR_GRAPH_PACKET_CAPTURE=1
run DEBUG_HIP_FORCE_GRAPH_QUEUES=1
run AMD_DIRECT_DISPATCH=0
run HIP_FORCE_DEV_KERNARG=1
run DEBUG_CLR_MAX_BATCH_SIZE=4096
run GPU_MAX_COMMAND_BUFFERS=64
