#!/bin/bash
# The CPU test suite's host-library tests (sampler, CPython-set emulation,
# graph builder, extend_nodes, pack code) against the ASan + UBSan build of
# host/*.cpp.  Python is not instrumented: libasan is preloaded, leaks off
# (the interpreter's own allocations are not ours to judge).
set -eo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
make -C "$ROOT/graphsage-pytorch_amd/csrc" sanitize >/dev/null
export GS_HOST_ASAN_LIB=$ROOT/graphsage-pytorch_amd/csrc/build/asan/libgraphsage_host_asan.so
export LD_PRELOAD="$(gcc -print-file-name=libasan.so) $(gcc -print-file-name=libubsan.so)"
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:halt_on_error=1
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
cd "$ROOT"
python -m pytest -q -p no:cacheprovider -m "not gpu" tests/test_host_sampler.py tests/test_unsup_native.py \
    --deselect tests/test_host_sampler.py::test_library_exports_every_declared_symbol "$@"
