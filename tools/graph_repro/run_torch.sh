#!/usr/bin/env bash
# Torch-level repro in both HIP graph capture modes (fresh processes: HIP reads the variable once).
cd "$(dirname "$0")"
DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 timeout -k 5 120 python -u torch_repro.py
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 5 120 python -u torch_repro.py
exit 0
