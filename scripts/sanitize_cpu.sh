#!/bin/bash
# the CPU test suite's oracle and host-runtime paths under AddressSanitizer +
# UndefinedBehaviorSanitizer (host code only; no GPU).  Builds both sanitized libraries with ROCm's
# clang (one shared sanitizer runtime), preloads that runtime into python, and runs the CPU tests
# that exercise them: the oracle (golden frames, KATs, sky, convention bounds use the plain variants),
# the host runtime's CPU paths (VariableManager TCP parsing incl. malformed packets, the recorder's
# conversion and sample times, host setTargetDepths, the noise-table generator, ABI exports).
# Any sanitizer report aborts the run (halt_on_error / -fno-sanitize-recover).
set -e
cd "$(dirname "$0")/.."
make -s -C oracle asan
make -s -C gpgpuraytrace_amd/csrc all asan
RT=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
export LD_PRELOAD="$RT"
export LD_LIBRARY_PATH="$(dirname "$RT"):/opt/rocm/lib/llvm/lib:${LD_LIBRARY_PATH}"
# python itself is not instrumented: its allocations are not leaks of ours
export ASAN_OPTIONS="detect_leaks=0:halt_on_error=1:abort_on_error=1:allocator_may_return_null=1"
export UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1"
python3 tests/tools/sanitize_run.py -q -p no:cacheprovider -m "not gpu" \
  tests/test_oracle.py tests/test_sky_kat.py tests/test_host.py tests/test_varmgr.py tests/test_output.py \
  tests/test_flyby.py "$@"
