for b in bin_phase bin_phase_lb bin_phase bin_phase_lb; do timeout -k 10 100 ./scripts/dbg/$b 20 0 > gpurun_out/ab_$b.txt 2>&1; echo "$b rc=$?"; cat gpurun_out/ab_$b.txt; done
