set -o pipefail
mkdir -p gpurun_out
for rb in 4 8; do
for g in 64 99 128; do
KFAC_EIG_RB=$rb KFAC_EIG_PROF=1 KFAC_EIG_G=$g timeout -k 10 120 python tools/bench_eig.py 785 > gpurun_out/eigrb.log 2>&1 || { tail -5 gpurun_out/eigrb.log; exit 1; }
echo "RB=$rb G=$g $(grep 'us/step' gpurun_out/eigrb.log | tail -1 | cut -c20-)"
done
done
