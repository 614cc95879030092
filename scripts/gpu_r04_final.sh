#!/bin/bash
# Round-4 closing check on the committed build: the GPU suite, smoke() and the default bench line.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/final_suite.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final_smoke.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/final_default_bench.json 2> gpurun_out/final_default_bench.err
echo "final rc=$?"
