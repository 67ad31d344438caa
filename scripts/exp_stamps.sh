set -o pipefail
cd /root/repo
mkdir -p gpurun_out/exp1
for v in stamps exp_NOCAS exp_NOADD exp_NOADD+NOCAS; do
  GS_STAMPS_LIB=libgossip_engine_$v.so timeout -k 10 200 python3 -u scripts/stamps.py > gpurun_out/exp1/$v.txt 2>&1 || exit 1
done
echo ok
