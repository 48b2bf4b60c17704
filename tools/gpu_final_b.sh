#!/bin/bash
# Round-end GPU pass, part B: kernel traces (two-stream and serialised), the stream timeline, PMC traffic and SQ
# passes, and the bench line carrying the measured traffic.  $1 = tag
TAG=${1:-r05}
SKIP_PYTEST=1 bash tools/gpu_round.sh $TAG
