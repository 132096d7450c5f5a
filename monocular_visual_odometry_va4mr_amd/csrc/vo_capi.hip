// Library-level C ABI entry points of libvo_hip.so (see include/vo_hip.h).
#include "vo_dev.h"

#include <string.h>

extern "C" const char* vo_version(void) { return "vo_hip 0.1 (gfx950)"; }

extern "C" int vo_device_cus(void)
{
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess) return VO_EHIP;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return VO_EHIP;
    return n;
}

// launch-shape threshold override (vo_set_launch_cus; read by device_cus() in vo_dev.h)
int vo_launch_cus_override = 0;

extern "C" int vo_set_launch_cus(int n)
{
    if (n < 0) return VO_EARG;
    vo_launch_cus_override = n;
    return VO_OK;
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

extern "C" int vo_stream_create_cumask(int reserve, int stride, vo_stream_t* out)
{
    if (!out || reserve < 0 || stride < 1) return VO_EARG;
    const int n = vo_device_cus();
    if (n <= 0) return VO_EHIP;
    if ((int64_t)reserve * stride > n) return VO_EARG;
    uint32_t mask[32];
    const int words = (n + 31) / 32;
    if (words > 32) return VO_EARG;
    memset(mask, 0, sizeof mask);
    for (int i = 0; i < n; ++i) mask[i >> 5] |= 1u << (i & 31);
    for (int k = 0; k < reserve; ++k) {
        const int i = stride - 1 + k * stride;
        mask[i >> 5] &= ~(1u << (i & 31));
    }
    hipStream_t st = nullptr;
    if (hipExtStreamCreateWithCUMask(&st, (uint32_t)words, mask) != hipSuccess) return VO_EHIP;
    *out = (vo_stream_t)st;
    return VO_OK;
}

extern "C" int vo_stream_destroy(vo_stream_t stream)
{
    return hipStreamDestroy((hipStream_t)stream) == hipSuccess ? VO_OK : VO_EHIP;
}
