#!/bin/bash
# Round-6 HEAD validation, part B: rocprofv3 kernel stats (B = 200 / 8192), PMC passes, roofline tables.
bash tools/gpu_profiles.sh ${1:-r6final}
