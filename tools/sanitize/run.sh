#!/bin/bash
# Host-side AddressSanitizer + UndefinedBehaviorSanitizer pass (SURVEY.md §5 sanitizer row):
# the product library rebuilt with the sanitizers on its HOST code only (-Xarch_host: the
# finishing adds of host_arith.hpp / G16Finish, gm_jac_*, the Horner tail, par_memcpy, the
# stage record gathering, pk dump / cache parsing), then the CPU tests that call into it,
# with the clang ASan runtime preloaded.  GPU code is not instrumented (not available on
# this pool).  Run here (no GPU):  bash tools/sanitize/run.sh
set -o pipefail
cd "$(dirname "$0")/../.."
ROOT=$PWD
B=gnark-icicle_amd/build_san
SAN="-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-omit-frame-pointer -Xarch_host -fno-sanitize-recover=undefined"
make -s -j${JOBS:-8} -C gnark-icicle_amd BUILD=build_san LIB=build_san/libgnark_mi355x.so TLIB=build_san/libgnark_mi355x_testhooks.so EXTRA="$SAN -g" build_san/libgnark_mi355x.so || exit 1
RT=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
export GNARK_MI355X_LIB=$ROOT/$B/libgnark_mi355x.so
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:halt_on_error=1
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
LD_PRELOAD=$RT timeout -k 10 900 python -m pytest -x -q -p no:cacheprovider \
  tests/test_capi_symbols.py tests/test_multirank.py tests/test_sanitize_host.py -m "not gpu" "$@"
