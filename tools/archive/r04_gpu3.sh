#!/bin/bash
# round 4: the config-5 PMC record, then config 3's shadow-pass A/B with LDS counters
cd "$(dirname "$0")/.."
timeout -k 10 900 bash tools/archive/r04_pmc5.sh && timeout -k 10 900 bash tools/archive/r04_shadow.sh
