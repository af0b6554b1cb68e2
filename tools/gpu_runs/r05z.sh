# Launch API comparison: hipLaunchKernel vs hipModuleLaunchKernel with one
# argument buffer (tools/launch_probe.hip, last rows).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05z; mkdir -p $O
timeout -k 10 240 tools/launch_probe 3000 > $O/launch_probe.jsonl 2> $O/launch_probe.err || { echo PROBE FAIL; cat $O/launch_probe.err; exit 1; }
grep '"launch"' $O/launch_probe.jsonl
