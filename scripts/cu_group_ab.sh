# A/B of k_iter's CU tile grouping (GQMAP_CU_GROUP=n overrides the occupancy-derived group; >=100 = whole band)
for r in 1 2; do for p in fp32 fp64; do for g in 1 3 4 100; do
  echo "mixture $p g$g: $(GQMAP_CU_GROUP=$g timeout -k 10 100 python scripts/prof_iter.py 200 $p mixture | grep -o 'graph run [0-9.]* us/it.*chk=[^ ]*')"
done; done; done
for g in 1 2 100; do
  echo "super fp64 g$g: $(GQMAP_CU_GROUP=$g timeout -k 10 100 python scripts/prof_iter.py 100 fp64 super | grep -o 'graph run [0-9.]* us/it')"
done
