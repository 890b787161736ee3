export TMPDIR=/tmp
tools/pmc.sh D r03dcol && tools/pmc_issue.sh Ddcol --workload D --steps 5 --warmup 1
