bash tools/lease.sh r6n "tests:multiprocess or inkernel or rmin or ranks or c4"; bash tools/ab_lib.sh 1 cur=-; BL_RMIN=1 bash tools/ab_lib.sh 1 rmin=-
