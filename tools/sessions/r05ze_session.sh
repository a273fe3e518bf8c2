#!/bin/bash
# cfg5's 8 shards at full size on one GPU with the final build (decode sweep): every repaired chunkset checked
set -o pipefail
export TMPDIR=/tmp
bash tools/cfg5_rehearsal.sh gpurun_out/r05ze/cfg5_rehearsal.jsonl 10 && python3 -c "
import json
for l in open('gpurun_out/r05ze/cfg5_rehearsal.jsonl'):
    d=json.loads(l); b=d['breakdown']; print(d['rehearsal'], d['value'], round(d['roofline']['frac'],4), round(d['roofline']['decode']['frac'],4), b['ready_chunksets'], b['not_ready_chunksets'])"
