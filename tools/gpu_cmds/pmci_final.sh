tools/gpu_session.sh \
 "pmci_D::400::bash tools/pmc_issue.sh D_r02f --workload D --steps 2 --warmup 1" \
 "pmci_B::200::bash tools/pmc_issue.sh B_r02f --workload B --steps 3 --warmup 1"
