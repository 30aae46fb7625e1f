#!/bin/bash
# Deeper narrow chunks on the rank shares (TTS_DEEP_LEVELS / TTS_DEEP_P3 / TTS_DEEP_P4)
set -o pipefail
run() { echo "== $*"; env "$@" timeout -k 10 300 python -u scripts/share_solve_probe.py 30 2>&1 | grep -v amdgpu || exit 1; }
run TTS_DEEP_LEVELS=2
run TTS_DEEP_LEVELS=3 TTS_DEEP_P3=4
run TTS_DEEP_LEVELS=3 TTS_DEEP_P3=12
run TTS_DEEP_LEVELS=4 TTS_DEEP_P3=12 TTS_DEEP_P4=2
run TTS_DEEP_LEVELS=4 TTS_DEEP_P3=12 TTS_DEEP_P4=4
