#!/bin/bash
# round 4: timeline of the 1/8 share, then the config-5 PMC record, then
# config 3's shadow-pass A/B with LDS counters (each script limits its steps)
cd "$(dirname "$0")/.."
timeout -k 10 400 bash tools/archive/r04_timeline.sh && timeout -k 10 900 bash tools/archive/r04_pmc5.sh && timeout -k 10 900 bash tools/archive/r04_shadow.sh
