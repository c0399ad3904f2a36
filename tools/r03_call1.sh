bash tools/r03_check.sh && NOPMC=1 bash tools/r03_slab.sh
