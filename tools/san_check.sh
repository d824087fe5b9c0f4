#!/bin/bash
# Host sanitizer runs, in this container (no GPU):
#  1. ASan + UBSan: libtmpt.so's host code (make SAN=1 -> _lib_san/: the threaded OBJ
#     parse and PNG encode, the octree build on 8 threads, the ABI's host hooks) and the
#     oracle (make SAN=1 -> oracle/build_san/: its pthreads render and batch HitScene),
#     loaded by the CPU tests that drive them;
#  2. TSan: tools/san_driver.cpp, the same host code and the oracle linked into one
#     program built with -fsanitize=thread, every threaded path run and checked against
#     its sequential form.
# Usage: tools/san_check.sh [log]   (exit status 0 = clean)
set -o pipefail
cd "$(dirname "$0")/.."
LOG=${1:-/dev/stdout}
CLANG=/opt/rocm/lib/llvm/bin/clang++
RT=$($CLANG -print-file-name=libclang_rt.asan-x86_64.so)
{
echo "== host sanitizers $(date -u +%FT%TZ), $($CLANG --version | head -1)"
make -s -C toymeshpathtracer_amd/csrc SAN=1 -j8 >/dev/null && make -s -C oracle SAN=1 >/dev/null || exit 1
echo "== 1. ASan + UBSan: CPU tests against _lib_san/libtmpt.so and oracle/build_san/liboracle.so"
LD_PRELOAD=$RT ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:detect_odr_violation=0 \
  UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 TMPT_NO_TORCH=1 \
  TMPT_LIB_PATH=$PWD/toymeshpathtracer_amd/_lib_san/libtmpt.so ORACLE_LIB=$PWD/oracle/build_san/liboracle.so \
  python -m pytest -q -p no:cacheprovider tests/test_host.py tests/test_octree.py tests/test_oracle.py \
    tests/test_octree_kat.py tests/test_abi.py -m "not gpu" -k "not header_compiles_as_c" 2>&1 || exit 1
echo "== 2. TSan: tools/san_driver.cpp"
mkdir -p tools/_bin
S=toymeshpathtracer_amd/csrc
CXX=/opt/rocm/lib/llvm/bin/clang++
CC=/opt/rocm/lib/llvm/bin/clang
HOSTINC="-D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -Iinclude -I$S"  # host-only: the HIP headers' host side
build_driver() {  # $1 = output, $2.. = sanitizer flags
    local out=$1; shift
    $CC -O1 -g -std=gnu11 -ffp-contract=off "$@" -c oracle/tmpt_oracle.c -o $out.oracle.o &&
    $CXX -O1 -g -std=c++17 -ffp-contract=off "$@" $HOSTINC -o $out tools/san_driver.cpp $S/tmpt_host.cpp \
        $S/tmpt_octree.cpp $out.oracle.o -lz -lpthread -lm
}
build_driver tools/_bin/san_driver_tsan -fsanitize=thread || exit 1
TSAN_OPTIONS=halt_on_error=1:second_deadlock_stack=1 tools/_bin/san_driver_tsan data 2>&1 || exit 1
echo "== 3. ASan + UBSan: the same driver"
build_driver tools/_bin/san_driver_asan -fsanitize=address,undefined -fno-sanitize-recover=undefined || exit 1
ASAN_OPTIONS=abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 tools/_bin/san_driver_asan data 2>&1 || exit 1
echo "== clean"
} > "$LOG" 2>&1
