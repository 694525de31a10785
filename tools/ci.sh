#!/bin/bash
# CI entry (the reference's CI only configured; this one builds and tests).
#   tools/ci.sh cpu   build everything (tools/build.py + CMake), native tests, sanitizer runs,
#                     CPU pytest (gloo multi-process, runtime, apps, models, fault tolerance)
#   tools/ci.sh gpu   GPU pytest on an MI355X (kernels vs fp32 references, models, 2-rank GPU
#                     data plane), smoke step and a short bench
set -eo pipefail
cd "$(dirname "$0")/.."
case "${1:-cpu}" in
  cpu)
    python tools/build.py
    python tools/lint.py
    cmake -S . -B build/cmake -G Ninja -DMINIPS_BUILD_KERNELS=OFF > /dev/null
    cmake --build build/cmake -j "${MAX_JOBS:-8}" > /dev/null
    ctest --test-dir build/cmake --output-on-failure
    ./build/bin/runtime_test
    python -m pytest tests -m "not gpu" -x -q
    ;;
  gpu)
    export HSA_ENABLE_IPC_MODE_LEGACY=0
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()"
    timeout -k 10 300 python bench.py --steps 20 --warmup 5
    ;;
  *) echo "usage: $0 cpu|gpu" >&2; exit 2 ;;
esac
