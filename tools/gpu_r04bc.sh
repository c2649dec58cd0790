#!/bin/bash
bash tools/gpu_r04b.sh; echo "r04b rc=$?"; bash tools/gpu_r04c.sh; echo "r04c rc=$?"
