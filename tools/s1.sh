source tools/gpu_steps.sh
run 300 smoke python __graft_entry__.py smoke
run 900 pytest_gpu python -m pytest tests -m gpu -q -x --timeout 600 -p no:cacheprovider
run 300 bench python bench.py --steps 200 --warmup 20
