// Drop-in for /root/reference/sift_cuda/types/CudaSiftConfig.hh:3-14.
// Field names (including the reference's spellings) and defaults are kept;
// the two trailing fields are additions with neutral defaults.
#pragma once

struct CudaSiftConfig {
    int col_width{0};            // image width in pixels
    int row_width{0};            // image height in pixels
    int numFeatures{5000};       // retainBest count (OpenCV nfeatures); 0 = keep all
    int numOctaveLayers{3};      // DoG layers scanned per octave
    double contrastThreshould{0.04};
    double edgeThreshould{10};
    double sigma{1.6};
    bool upscale{false};         // true = OpenCV default firstOctave -1 (works here)
    int numOctaves{0};           // 0 = auto: cvRound(log2(min(W,H)) - 2) - firstOctave
    int maxKeypoints{0};         // result capacity; 0 = sized from numFeatures / the frame (sift_hip.h)
};
