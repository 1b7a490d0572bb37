// The fp32 kernel for models wider than 512 (up to 1024; see ik_ann.hip,
// launch_ann_wide), compiled with 1028-float LDS rows and 32-point tiles.
#define IKHIP_ANN_WIDE 1
#include "ik_ann.hip"
