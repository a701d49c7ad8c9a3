#!/bin/bash
cd "$GRAFT_REPO_ROOT"
for f in 0 1 2 4 7; do echo "fold-off bits $f"; TTS_DEBUG_FOLD=$f timeout -k 10 120 python3 scripts/debug_dia.py 2>&1 | grep -E "hd64|wide1" || exit 1; done
