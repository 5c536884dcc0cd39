cd $GRAFT_REPO_ROOT
for cfg in "" "HF3FS_CRC_SYNC_FREE=1" "HF3FS_CRC_NO_POOL=1" "" "HF3FS_CRC_STATIC=1"; do
  env $cfg timeout -k 10 120 ./tests/cpp/test_checksuminfo > gpurun_out/cpp_b.log 2>&1; rc=$?
  echo "cfg=[$cfg] rc=$rc $(tail -1 gpurun_out/cpp_b.log) $(grep -m1 -A2 'mode=' gpurun_out/cpp_b.log | tr '\n' ' ')"
  if [ $rc -gt 1 ]; then exit $rc; fi
done
