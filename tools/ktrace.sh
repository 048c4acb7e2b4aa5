# kernel-trace summary of one bench configuration: tools/ktrace.sh NAME [bench args...]
set -e
name=$1; shift
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/kt_$name -o run -- python3 $GRAFT_REPO_ROOT/bench.py --quick "$@" > $GRAFT_REPO_ROOT/gpurun_out/kt_$name.log 2>&1
