bash tools/gpu_r03e.sh r03e && bash tools/gpu_ab_small.sh r03f eagerp xd16 xe1
