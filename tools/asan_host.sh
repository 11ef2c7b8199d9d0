#!/bin/bash
# Host AddressSanitizer run of the C-ABI layer (CPU only; GPU sanitizers are not available on the
# pool): builds the library with the host halves of every .hip file instrumented
# (-Xarch_host -fsanitize=address; device code unchanged) into /tmp, then runs the host ABI tests
# (symbol exports, struct layout, workspace queries, null / zero arguments of every entry point)
# against it with the ASan runtime preloaded.  usage: tools/asan_host.sh
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
W=/tmp/unet_asan
rm -rf $W && mkdir -p $W/a/b
cp -r "$ROOT/unet-image-segmentation_amd/csrc" $W/a/b/csrc
cp -r "$ROOT/include" $W/a/include
make -C $W/a/b/csrc -j8 OUT=$W/libunet_hip_asan.so \
  HIPFLAGS="-O1 -g -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-result -ffp-contract=fast -Xarch_host -fsanitize=address -Xarch_host -fno-omit-frame-pointer"
RT=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
cd "$ROOT"
ASAN_OPTIONS=detect_leaks=0 LD_PRELOAD=$RT UNET_HIP_LIB=$W/libunet_hip_asan.so \
  python -m pytest tests/test_abi_host.py -q -p no:cacheprovider
