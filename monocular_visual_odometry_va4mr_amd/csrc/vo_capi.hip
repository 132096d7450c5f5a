// Library-level C ABI entry points of libvo_hip.so (see include/vo_hip.h).
#include "vo_dev.h"

#include <string.h>

extern "C" const char* vo_version(void) { return "vo_hip 0.1 (gfx950)"; }

// A stream whose kernels only start workgroups on the CUs set in `mask` (bit i of word i/32 =
// CU i).  The engine puts its bulk single-wave launches (LK) on one, so the large latency-bound
// workgroups of the other stream group always find free CUs (overlap).
extern "C" int vo_stream_create_cumask(int nwords, const uint32_t* mask, vo_stream_t* out)
{
    if (!mask || !out || nwords <= 0) return VO_EARG;
    hipStream_t s = nullptr;
    if (hipExtStreamCreateWithCUMask(&s, (uint32_t)nwords, mask) != hipSuccess) return VO_EHIP;
    *out = (vo_stream_t)s;
    return VO_OK;
}

extern "C" int vo_stream_destroy(vo_stream_t s)
{
    if (!s) return VO_EARG;
    return hipStreamDestroy((hipStream_t)s) == hipSuccess ? VO_OK : VO_EHIP;
}

extern "C" int vo_device_cus(void)
{
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess) return VO_EHIP;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return VO_EHIP;
    return n;
}

extern "C" int vo_device_arch(char* buf, int len)
{
    if (!buf || len <= 0) return VO_EARG;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return VO_EHIP;
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, dev) != hipSuccess) return VO_EHIP;
    strncpy(buf, p.gcnArchName, (size_t)len - 1);
    buf[len - 1] = 0;
    return VO_OK;
}
