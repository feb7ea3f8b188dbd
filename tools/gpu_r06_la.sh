#!/bin/bash
# Round 6: the plugin's look-ahead through hl_codec_encode (tools/per_frame_api.py):
# 120 frames of the bench stream one by one, and with a 20-frame look-ahead.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/per_frame_api.py 120 bench_1088p_s11 1 > gpurun_out/r06_la_api.log 2>&1 || { tail -3 gpurun_out/r06_la_api.log; exit 1; }
for k in 8 20 60; do
  timeout -k 10 300 python3 -u tools/per_frame_api.py 120 bench_1088p_s11 $k >> gpurun_out/r06_la_api.log 2>&1 || { tail -3 gpurun_out/r06_la_api.log; exit 1; }
done
grep '^{' gpurun_out/r06_la_api.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d.get('lookahead',1), d['bitexact'], d.get('all_fps'), d.get('mean_p_ms'), d.get('all_ms'))"
