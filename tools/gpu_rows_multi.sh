bash tools/gpu_rows_ablate.sh aligned noload dwords x3 nolut w8 && KNOBS="AEON_HIP_ROWS_TR=38" bash tools/gpu_rows_ablate.sh w8 nolut
KNOBS="AEON_HIP_ROWS_DEVJOBS=1" bash tools/gpu_rows_ablate.sh w8
