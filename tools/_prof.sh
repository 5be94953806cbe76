set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for cfg in sift1m gist1m deep10m; do
  timeout -k 10 500 bash tools/profile_box.sh r01_$cfg --config $cfg > gpurun_out/prof_$cfg.log 2>&1 || { echo "profile $cfg failed"; tail -20 gpurun_out/prof_$cfg.log; exit 1; }
  echo "profiled $cfg"
done
