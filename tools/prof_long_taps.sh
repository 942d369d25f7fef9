set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/lt
mkdir -p $O
timeout -k 10 60 rocprofv3 -L > $O/avail.txt 2>&1 || true
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU --kernel-trace -d $O/sqa -o run --output-format csv -- python tools/long_taps_one.py 31 i16u8 6 > $O/sqa.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/fetch -o run --output-format csv -- python tools/long_taps_one.py 31 i16u8 6 > $O/fetch.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/write -o run --output-format csv -- python tools/long_taps_one.py 31 i16u8 6 > $O/write.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d $O/stats -o run --output-format csv -- python tools/long_taps_one.py 31 i16u8 30 > $O/stats.log 2>&1 || exit 1
echo done
