#!/bin/bash
bash scripts/gpu_sq.sh sq gemm 128 && bash scripts/gpu_sq.sh sq direct 128
