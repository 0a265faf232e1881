bash tools/gpu_seg_debug.sh base && bash tools/sq_seg_variants.sh base po ma
