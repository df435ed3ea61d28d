#!/bin/bash
# Host-only tools linked against anothertls_amd/libatls.so (built by __graft_entry__.build()).
set -e
cd "$(dirname "$0")/.."
g++ -O2 -std=c++17 -Wall -Iinclude tools/c1_loopback_native.cpp -Lanothertls_amd -latls \
    -Wl,-rpath,'$ORIGIN/../anothertls_amd' -lpthread -o tools/c1_loopback_native
# RCCL point-to-point size probe (tools/rccl_p2p_probe.cpp)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O2 -std=c++17 -I/opt/rocm/include tools/rccl_p2p_probe.cpp -ldl \
    -o tools/rccl_p2p_probe
# Single-call latency floors (tools/single_call_floor.hip)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O2 -std=c++17 -Iinclude tools/single_call_floor.hip -Lanothertls_amd -latls \
    -Wl,-rpath,'$ORIGIN/../anothertls_amd' -o tools/single_call_floor
