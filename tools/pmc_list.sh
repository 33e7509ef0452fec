set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > gpurun_out/pmc_list.txt 2>&1; echo "LIST $?"
grep -oE "(SQC?_[A-Z_0-9]+|TCP_[A-Z_0-9]+|TCC_[A-Z_0-9]+)" gpurun_out/pmc_list.txt | sort -u > gpurun_out/pmc_names.txt; wc -l gpurun_out/pmc_names.txt
