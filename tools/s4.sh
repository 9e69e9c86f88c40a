source tools/gpu_steps.sh
export TMPDIR=/tmp
R=$PWD
run 300 probe python tools/probe_rollout.py --B 2048,4096,8192,16384 --N 200
run 300 probe_misc python tools/probe_rollout.py --B 4096 --N 200 --scheme naive
run 300 probe_ph python tools/probe_rollout.py --B 4096 --N 200 --philox
run 900 pytest_gpu python -m pytest tests -m gpu -q -x --timeout 600 -p no:cacheprovider
