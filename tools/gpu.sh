#!/bin/bash
# Runs a command on the GPU box via gpurun (one call, no retries) and prints
# the tail of its output.  Usage:
#   tools/gpu.sh TIMEOUT 'command'
t=$1; shift
/usr/local/graft/bin/gpurun --timeout "$t" -- "$@" 2>&1 | tail -25
