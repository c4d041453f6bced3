#!/bin/bash
# The fourth-stream A/B (gpu_r04s.sh), then the C5 bench line (gpu_r04r.sh).
bash scripts/gpu_r04s.sh && bash scripts/gpu_r04r.sh
