#!/bin/bash
bash tools/gpu_r4_k.sh && bash tools/gpu_r4_l.sh
