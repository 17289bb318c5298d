#!/bin/bash
# Builds build/bin/exit_order_probe (+ build/lib/libexit_order_dep.so).
set -e
cd "$(dirname "$0")/../.."
mkdir -p build/bin build/lib
g++ -O2 -shared -fPIC tools/exit_order/probe_dep.cpp -o build/lib/libexit_order_dep.so
hipcc --offload-arch=gfx950 -O2 tools/exit_order/probe.hip -o build/bin/exit_order_probe \
  -Wl,--no-as-needed -Lbuild/lib -lexit_order_dep -Wl,-rpath,'$ORIGIN/../lib'
