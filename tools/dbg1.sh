set -o pipefail
cd $GRAFT_REPO_ROOT
o=gpurun_out/dbg1.log
timeout -k 10 200 python -u tools/debug_batch.py 4 50000 5000 52 50000 5000 256 50000 5000 > $o 2>&1 || { tail $o; exit 1; }
FLEETPLACE_PIPE_W=4 FLEETPLACE_PIPE_SEG=40 timeout -k 10 100 python -u tools/debug_batch.py 4 50000 5000 >> $o 2>&1 || { tail $o; exit 1; }
FLEETPLACE_PIPE_W=4 FLEETPLACE_PIPE_SEG=4 timeout -k 10 100 python -u tools/debug_batch.py 256 50000 5000 >> $o 2>&1 || { tail $o; exit 1; }
FLEETPLACE_LIB=$PWD/fleetflow_amd/libfleetplace_noasm.so timeout -k 10 100 python -u tools/debug_batch.py 256 50000 5000 52 50000 5000 >> $o 2>&1 || { tail $o; exit 1; }
cat $o
