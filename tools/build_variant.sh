#!/bin/bash
# Build an in-tree variant of libslam_hip.so with extra preprocessor flags
# (development tool): tools/build_variant.sh NAME "-DFLAG ..." -> slamhip/libslam_NAME.so
set -e
cd "$(dirname "$0")/../slam-robot_simu_amd"
name=$1; shift
mkdir -p build/var_$name
pids=()
for f in csrc/*.hip; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function $@ -c $f -o build/var_$name/$(basename ${f%.hip}).o &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -Wl,--no-undefined -o slamhip/libslam_$name.so build/var_$name/*.o
echo built slamhip/libslam_$name.so
