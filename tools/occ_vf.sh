for pad in 0 53000 80000; do
  for rep in 1 2; do
    echo "== pad $pad rep $rep" >> gpurun_out/occ.log
    GOL_BAND_VF=1 GOL_BAND_LDS_PAD=$pad timeout -k 10 120 python tools/sweep.py --rounds 2 --variants b:8:128:0 >> gpurun_out/occ.log 2>/dev/null || exit 3
  done
done
