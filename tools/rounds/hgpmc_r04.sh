set -u
bash tools/hashgrid_prof.sh gpurun_out/hgpmc15 --only 15 && bash tools/hashgrid_prof.sh gpurun_out/hgpmc0 --only 0 && \
python3 tools/pmc_summary.py hashgrid_bwd_kernel gpurun_out/hgpmc15/p1 gpurun_out/hgpmc15/p2 > gpurun_out/hgpmc15/summary.txt && \
python3 tools/pmc_summary.py hashgrid_bwd_kernel gpurun_out/hgpmc0/p1 gpurun_out/hgpmc0/p2 > gpurun_out/hgpmc0/summary.txt && cat gpurun_out/hgpmc15/summary.txt gpurun_out/hgpmc0/summary.txt
