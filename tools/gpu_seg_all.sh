bash tools/gpu_seg_debug.sh segguard base && bash tools/gpu_seg_try.sh seg4
