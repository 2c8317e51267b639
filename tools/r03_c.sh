#!/bin/bash
# r03_b (witness-program tests, configs[0] latency + timeline), then the
# round's bench + rocprof + PMC evidence (tools/profile_r02.sh r03).
set -e
bash tools/r03_b.sh
bash tools/profile_r02.sh r03
