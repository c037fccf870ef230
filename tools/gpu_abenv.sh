#!/bin/bash
# A/B of geometry env settings on the bench (no CPU baseline):
#   tools/gpu_abenv.sh <tag> "<name>:<ENV=V ENV2=V2>" ...   (empty env = defaults)
set -o pipefail
tag=${1:?tag}; shift
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out
for spec in "$@"; do
  name=${spec%%:*}; envs=${spec#*:}
  env $envs timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 3 --warmup 1 \
     > gpurun_out/${tag}_env_${name}.json 2> gpurun_out/${tag}_env_${name}.err || { echo "ab $name failed"; tail gpurun_out/${tag}_env_${name}.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'step', round(d['ms_per_step'],2), 'ffd', round(d['breakdown_ms']['ffd_kernel'],2), 'sort', round(d['breakdown_ms']['sort'],2), '| c3 step', round(d['config3']['ms_per_step'],2), 'ffd', round(d['config3']['breakdown_ms']['ffd_kernel'],2))" gpurun_out/${tag}_env_${name}.json "$name"
done
