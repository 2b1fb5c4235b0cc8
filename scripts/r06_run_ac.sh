set -u
O=${O:-gpurun_out/r6ac}
mkdir -p $O
timeout -k 10 300 python3 scripts/host_profile_single.py 200 > $O/host_profile.txt 2> $O/host_profile.err || exit $?
