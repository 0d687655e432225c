/*
 * fmgi_lds_attr.h -- raising a kernel's dynamic-LDS limit once per device (fold and radiosity kernels).
 */
#ifndef FMGI_LDS_ATTR_H
#define FMGI_LDS_ATTR_H

#include <hip/hip_runtime_api.h>
#include <stdint.h>

#include <atomic>
#include <mutex>
#include <set>
#include <utility>

/* hipFuncSetAttribute(MaxDynamicSharedMemorySize) once per (kernel, device): the attribute belongs to the
   device, so a process baking on several GPUs sets it on each (Tag tells the call sites' kernels apart;
   concurrent first calls just set it twice) */
template <int Tag>
inline hipError_t fmgi_set_lds_attr_once(const void *fn, int bytes) {
    static std::atomic<uint64_t> done{0};
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    const uint64_t bit = 1ull << (dev & 63);
    if (done.load(std::memory_order_acquire) & bit) return hipSuccess;
    e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    if (e == hipSuccess) done.fetch_or(bit, std::memory_order_acq_rel);
    return e;
}

/* the same for a kernel chosen at run time: once per (device, kernel) */
inline hipError_t fmgi_set_lds_attr_fn(const void *fn, int bytes) {
    static std::mutex mu;
    static std::set<std::pair<int, const void *>> done;
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    std::lock_guard<std::mutex> lk(mu);
    if (done.count({dev, fn})) return hipSuccess;
    e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    if (e == hipSuccess) done.insert({dev, fn});
    return e;
}

#endif
