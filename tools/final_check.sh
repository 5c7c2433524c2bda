set -e
mkdir -p gpurun_out/final
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/final/tests.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final/smoke.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/final/c2.log 2>&1
timeout -k 10 200 python bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline --no-serial > gpurun_out/final/c3.log 2>&1
timeout -k 10 200 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline --no-serial > gpurun_out/final/c5.log 2>&1
