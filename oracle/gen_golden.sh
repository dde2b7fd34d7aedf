#!/usr/bin/env bash
# TEST INFRASTRUCTURE ONLY: regenerate tests/golden/*.json from the reference
# build in oracle/_ref (see oracle/Makefile `golden`).  Run in the container
# that has /root/reference; the fixtures are committed and travel as data.
set -euo pipefail
cd "$(dirname "$0")"
out=../tests/golden
mkdir -p "$out"
./_ref/ref_golden_box --common > "$out/ref_box.json"
./_ref/ref_golden_box_mirror > "$out/ref_box_mirror.json"
./_ref/ref_golden_simple > "$out/ref_simple.json"
python3 -c "import json,sys; [json.load(open(f)) for f in sys.argv[1:]]" "$out"/ref_*.json
ls -l "$out"
