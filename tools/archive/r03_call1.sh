bash tools/archive/r03_check.sh && NOPMC=1 bash tools/archive/r03_slab.sh
