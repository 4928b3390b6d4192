#!/usr/bin/env bash
# tools/asan_build.sh — a host-AddressSanitizer build of libmec and of two
# host-side drivers, for runs on the GPU box (device code unchanged: every
# -fsanitize flag applies to the host side only, -Xarch_host).
#   memec_amd/asan/libmec.so      every csrc unit, host code instrumented
#   tools/coding_bench_asan       MemEC's calling pattern through the adapter
#   tools/queue_latency_asan      single-caller queue calls, traced
# The ASan runtime is linked statically into the two executables (clang's
# default), so no preload is involved.  Run with
#   ASAN_OPTIONS=detect_leaks=0:abort_on_error=1
set -eu
cd "$(dirname "$0")/.."
HIPCC=/opt/rocm/bin/hipcc
CLANG=/opt/rocm/llvm/bin/clang++
ASAN="-Xarch_host -fsanitize=address -Xarch_host -fno-omit-frame-pointer"
OUT=memec_amd/build_asan
LIB=memec_amd/asan
mkdir -p "$OUT" "$LIB"
FLAGS="--offload-arch=gfx950 --offload-compress -O2 -g -std=c++17 -fPIC -Wall -Iinclude -Imemec_amd/csrc $ASAN"
objs=()
pids=()
for f in memec_amd/csrc/*.hip memec_amd/csrc/*.cpp; do
    o="$OUT/$(basename "${f%.*}").o"
    objs+=("$o")
    # rebuilt when the source or any header is newer (a unit compiled
    # against an older ctx.hpp would disagree on mec_ctx's layout)
    stale=0
    [ ! -f "$o" ] || [ "$f" -nt "$o" ] && stale=1
    for h in memec_amd/csrc/*.hpp include/mec.h; do [ "$h" -nt "$o" ] && stale=1; done
    if [ $stale = 1 ]; then
        $HIPCC $FLAGS -c -o "$o" "$f" &
        pids+=($!)
        if [ ${#pids[@]} -ge 8 ]; then wait "${pids[0]}"; pids=("${pids[@]:1}"); fi
    fi
done
for p in "${pids[@]}"; do wait "$p"; done
$HIPCC --offload-arch=gfx950 -shared -fPIC -o "$LIB/libmec.so" "${objs[@]}" -Wl,-soname,libmec.so -L/opt/rocm/lib -lhiprtc -Wl,-rpath,/opt/rocm/lib
$CLANG -std=c++11 -O1 -g -fsanitize=address -fno-omit-frame-pointer -Imemec_amd/csrc/coding -Iinclude \
    tools/coding_bench.cc memec_amd/csrc/coding/*.cc -L"$LIB" -lmec -Wl,-rpath,'$ORIGIN/../memec_amd/asan' \
    -lpthread -o tools/coding_bench_asan
$HIPCC --offload-arch=gfx950 -O1 -g -std=c++17 -Iinclude $ASAN tools/queue_latency.hip -L"$LIB" -lmec \
    -Wl,-rpath,'$ORIGIN/../memec_amd/asan' -o tools/queue_latency_asan
echo "asan build done"
