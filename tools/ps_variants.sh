for v in stats v12r8 v13r4 v12r16; do
  echo "== $v"
  APE_LZ4_LIB=$PWD/libapenetwork_amd/libape_lz4_amd_$v.so timeout -k 10 200 python3 tools/phase_stats.py 16384 1 > gpurun_out/ps_$v.txt 2>&1 || exit 1
  grep -E "^encode|candidates|walk|emit|verified" gpurun_out/ps_$v.txt
done
