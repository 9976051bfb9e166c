#!/bin/bash
# Build libmpo.so's host code with AddressSanitizer (device code unchanged; the
# sanitizer flags go to the host compilation only) and run the host-side ABI
# driver under it.  No GPU needed.  Output: build/asan/ (git-ignored).
set -euo pipefail
cd "$(dirname "$0")/.."
B=mpi_opt_amd/csrc/build/asan
mkdir -p $B
HIPCC=/opt/rocm/bin/hipcc
SAN="-Xarch_host -fsanitize=address -Xarch_host -fno-omit-frame-pointer"
FLAGS="-O1 -g -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-result $SAN"
objs=""
for f in mpi_opt_amd/csrc/*.hip; do
  o=$B/$(basename $f .hip).o
  if [ ! -f $o ] || [ $f -nt $o ] || [ include/mpo.h -nt $o ]; then $HIPCC $FLAGS -c $f -o $o & fi
  objs="$objs $o"
done
$HIPCC $FLAGS -x hip -c mpi_opt_amd/csrc/api.cpp -o $B/api.o &
wait
$HIPCC -shared -fPIC --offload-arch=gfx950 -Xarch_host -fsanitize=address -o $B/libmpo_asan.so $objs $B/api.o
/opt/rocm/llvm/bin/clang++ -O1 -g -fno-gpu-sanitize -fsanitize=address -fno-omit-frame-pointer -std=c++17 tests/asan/abi_driver.cpp -o $B/abi_driver \
    -L$B -lmpo_asan -Wl,-rpath,$(pwd)/$B
# HIP's runtime keeps process-lifetime allocations: leak checking is off, every
# other ASan check (overflows, use-after-free, double free) is on
ASAN_OPTIONS=detect_leaks=0:abort_on_error=0 $B/abi_driver
