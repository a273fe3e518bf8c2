#!/bin/bash
# r05i (FETCH_SIZE calibration for 8-byte loads) then r05j (8-column decode variants), one box
set -o pipefail
bash tools/sessions/r05i_session.sh && bash tools/sessions/r05j_session.sh
