#!/usr/bin/env bash
cd "$(dirname "$0")" && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -shared -o fetch_calib.so fetch_calib.hip
