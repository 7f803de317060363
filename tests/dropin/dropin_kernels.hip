// Device half of the drop-in harness: the gfx950 kernels of the test-defined semirings
// (HipSpGEMMKernels.h), compiled with hipcc. The reference drivers run in dropin_harness.cpp.
#include "CombBLAS/CombBLAS.h"
#include "combblas_hip/HipSpGEMMKernels.h"
#include "dropin_semirings.h"

typedef combblas::PlusTimesSRing<double, int64_t> PTDI;
COMBBLAS_HIP_DEVICE_KERNELS(KTipsDev, int64_t, bool, bool, bool)
COMBBLAS_HIP_DEVICE_KERNELS(MinMaxDev, int64_t, int64_t, int64_t, MinMax)
COMBBLAS_HIP_DEVICE_KERNELS(PTDI, int64_t, double, int64_t, double)
typedef combblas::Select2ndSRing<int64_t, int64_t, int64_t> S2LL;
COMBBLAS_HIP_DEVICE_KERNELS(S2LL, int64_t, int64_t, int64_t, int64_t)
COMBBLAS_HIP_DEVICE_KERNELS(PTOrdDev, int64_t, double, double, double)
COMBBLAS_HIP_DEVICE_KERNELS(AffineDev, int64_t, double, double, double)
