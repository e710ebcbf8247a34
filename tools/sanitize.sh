#!/bin/bash
# Host sanitizer pass over the CPU test suite.
#
# Builds libsnpmi.so's host code with ASan+UBSan and with TSan (`make -C pysnptools_amd/csrc asan
# tsan`: -Xarch_host, the gfx950 device code is compiled as usual) and the oracle with gcc's
# ASan+UBSan (`make -C oracle asan`), then runs the CPU tests that drive the host code
# -- the threaded .fam/.bim parser (test_meta), the AVX2 host generator (test_host_synth), the
# multi-threaded mmap gather into pinned pieces / snpmi_bed_gather_packed and the C-ABI argument
# checks (test_api_host, test_abi), the oracle C (test_oracle) -- with the matching runtime
# preloaded into the (uninstrumented) Python.  One runtime per process: clang's for libsnpmi, gcc's
# for the oracle.  Logs go to $1 (default profiles/r06_sanitize); exit status != 0 on any report.
set -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=${1:-$ROOT/profiles/r06_sanitize}
mkdir -p "$OUT"
make -s -j8 -C "$ROOT/pysnptools_amd/csrc" asan tsan || exit 2
make -s -C "$ROOT/oracle" asan || exit 2
RT=$(ls -d /opt/rocm/lib/llvm/lib/clang/*/lib/linux | head -1)
GCC_ASAN=$(gcc -print-file-name=libasan.so)
SNPMI_TESTS="tests/test_meta.py tests/test_host_synth.py tests/test_api_host.py tests/test_abi.py tests/test_watchdog_host.py"
ORACLE_TESTS="tests/test_oracle.py"
cd "$ROOT" || exit 2
status=0
run() {  # name, tests, env assignments...
    local name=$1 tests=$2
    shift 2
    echo "== $name: $tests" | tee "$OUT/$name.log"
    # shellcheck disable=SC2086
    # -s: a sanitizer report is written to fd 2 as the process exits -- pytest's capture would eat it
    env "$@" python -c "import os; from pysnptools_amd import _native as N; from oracle import oracle as O; print('libsnpmi:', N.LIB_PATH, '| oracle:', os.environ.get('ORACLE_LIB', 'default'))" >>"$OUT/$name.log" 2>&1
    env "$@" python -m pytest -q -s -m "not gpu" -p no:cacheprovider $tests >>"$OUT/$name.log" 2>&1
    local rc=$?
    if grep -qE "ERROR: (AddressSanitizer|LeakSanitizer)|runtime error:|WARNING: ThreadSanitizer" "$OUT/$name.log"; then
        rc=99
    fi
    echo "rc=$rc" >>"$OUT/$name.log"
    tail -3 "$OUT/$name.log"
    [ $rc -eq 0 ] || status=1
}
run libsnpmi_asan_ubsan "$SNPMI_TESTS" LD_PRELOAD="$RT/libclang_rt.asan-x86_64.so" \
    ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:detect_odr_violation=0 \
    UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 \
    SNPMI_LIB="$ROOT/pysnptools_amd/csrc/build/asan/libsnpmi.so"
run libsnpmi_tsan "$SNPMI_TESTS" LD_PRELOAD="$RT/libclang_rt.tsan-x86_64.so" \
    TSAN_OPTIONS=halt_on_error=1:report_signal_unsafe=0 \
    SNPMI_LIB="$ROOT/pysnptools_amd/csrc/build/tsan/libsnpmi.so"
run oracle_asan_ubsan "$ORACLE_TESTS" LD_PRELOAD="$GCC_ASAN" \
    ASAN_OPTIONS=detect_leaks=0:halt_on_error=1 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 \
    ORACLE_LIB="$ROOT/oracle/_san/liboracle_asan.so"
# No TSan pass of the oracle: its threads are OpenMP's, and the image's libgomp is not built with
# TSan, so every parallel region's join is invisible to it (a run reports the loop's reads racing
# NumPy's later free of the output -- the known libgomp false positive); its loops write disjoint
# output columns.  libsnpmi's own threads are std::thread (parallel_for) and are covered above.
exit $status
