set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_abenv.sh r02e "ww3_seg32:" "ww3_seg20:FLEETPLACE_PIPE_SEG=20" "ww3_seg16:FLEETPLACE_PIPE_SEG=16" "ww2_seg32:FLEETPLACE_LIB=$PWD/fleetflow_amd/libfleetplace_ww2.so" "ww2_seg20:FLEETPLACE_LIB=$PWD/fleetflow_amd/libfleetplace_ww2.so FLEETPLACE_PIPE_SEG=20"
