// The bf16x6-mode instantiations of ann_fused_kernel (see ik_ann.hip,
// launch_ann_kernel_x), compiled apart from the fp32 kernel.
#define IKHIP_ANN_X_TU 1
#include "ik_ann.hip"
