# every pattern of capture_patterns.hip at 1, 2, 4, 50 iterations; stops at
# the first crash (a crash inside HIP's capture code: no GPU work involved)
for p in ${PATTERNS:-0 5 4 2 7 6 3 1}; do for n in ${NS:-1 2 4 50}; do timeout -k 5 30 ./scripts/micro/capture_patterns $p $n; rc=$?; echo "pattern $p n $n rc $rc"; if [ $rc -ge 124 ]; then exit 0; fi; done; done
