set -u
cd /root/repo
timeout -k 10 120 python -u tools/uvec_check.py > gpurun_out/uvec_check.txt 2>&1; rc=$?; cat gpurun_out/uvec_check.txt | grep uvec; [ $rc -le 1 ] || exit $rc
for c in "encode104 2" "decode104 2" "encode83 4100"; do set -- $c
  timeout -k 10 120 python -u tools/tune.py --config $1 --pad $2 --rounds 5 --iters 10 --variants ";uvec=1" > gpurun_out/uvec_$1.txt 2>&1 || exit $?
  grep frac gpurun_out/uvec_$1.txt | sed "s/^/$1 /"
done
