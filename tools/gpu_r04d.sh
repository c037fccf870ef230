set -o pipefail
tools/ab_variants.sh r04d "- _sb" c4x4096,c4x512,c3 || exit 1
FLEETPLACE_LIB=$PWD/fleetflow_amd/libfleetplace_stats.so timeout -k 10 200 python -u tools/pipe_stats.py 4096 > gpurun_out/r04d_stats_c4.txt 2>&1 || exit 1
FLEETPLACE_LIB=$PWD/fleetflow_amd/libfleetplace_stats.so C=1000000 N=100000 SEED=0x5EED0003 SPAN=gpurun_out/r04d_span_c3.csv timeout -k 10 200 python -u tools/pipe_stats.py 1 > gpurun_out/r04d_stats_c3.txt 2>&1 || exit 1
cat gpurun_out/r04d_stats_c4.txt gpurun_out/r04d_stats_c3.txt
