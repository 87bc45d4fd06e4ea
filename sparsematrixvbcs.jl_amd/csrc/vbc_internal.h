// Internal helpers shared by the host and device translation units of libvbc.
#pragma once
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

#include "vbc.h"

namespace vbc {

// Thread-local last-error message (vbc_last_error).
void set_error(const char *fmt, ...) __attribute__((format(printf, 1, 2)));

inline int fail(int status, const char *what)
{
    set_error("%s", what);
    return status;
}

// Environment knobs read at create time.
//  * layout_knob: a layout choice.  Every value selects a layout that the -m gpu
//    parity tests hold to the oracle; none changes what a product computes beyond the rounding that
//    vbc.h states for the split layouts (VBC_CREATE_SERIAL forbids those).
//  * tuning_knob: a launch / layout tuning constant (range counts, pipeline depths, thresholds) that the
//    product library keeps at its measured default; the VBC_ABLATION build reads it for tools/ab.py sweeps.
//  * ablation_knob / VBC_ABL: ablation variants that time a kernel with part of its work removed (x
//    taken as 1, gathers confined to a few lines, stores dropped): wrong products by design.  Only the
//    -DVBC_ABLATION build reads them and instantiates those kernels (`make ablation` ->
//    tools/exp/libs/libvbc_ablation.so, for tools/ab.py); the product libvbc.so does neither.
inline const char *layout_knob(const char *name) { return std::getenv(name); }
#ifdef VBC_ABLATION
#define VBC_ABL(expr) (expr)
inline const char *ablation_knob(const char *name) { return std::getenv(name); }
inline const char *tuning_knob(const char *name) { return std::getenv(name); }
#else
#define VBC_ABL(expr) 0
inline const char *ablation_knob(const char *) { return nullptr; }
inline const char *tuning_knob(const char *) { return nullptr; }
#endif

inline int elem_size(int dtype)
{
    switch (dtype) {
    case VBC_F64: case VBC_I64: return 8;
    case VBC_F32: case VBC_I32: return 4;
    case VBC_BOOL: return 1;
    default: return 0;
    }
}

// Strided host vector of eltype `dt` (vbc_dtype) converted to a contiguous To[n] (Julia's convert).
template <typename To>
void host_convert(const void *src, int dt, int64_t n, int64_t inc, To *dst)
{
    const char *p = static_cast<const char *>(src);
    for (int64_t i = 0; i < n; i++) {
        const char *e = p + i * inc * elem_size(dt);
        switch (dt) {
        case VBC_F64: dst[i] = (To) * reinterpret_cast<const double *>(e); break;
        case VBC_F32: dst[i] = (To) * reinterpret_cast<const float *>(e); break;
        case VBC_I64: dst[i] = (To) * reinterpret_cast<const int64_t *>(e); break;
        case VBC_I32: dst[i] = (To) * reinterpret_cast<const int32_t *>(e); break;
        default: dst[i] = (To) * reinterpret_cast<const uint8_t *>(e); break;
        }
    }
}

// The same into a contiguous vector of the compute eltype cdt (F64 / F32 / I64).
inline void host_convert_to(const void *src, int dt, int64_t n, int64_t inc, void *dst, int cdt)
{
    if (cdt == VBC_F64) host_convert(src, dt, n, inc, static_cast<double *>(dst));
    else if (cdt == VBC_F32) host_convert(src, dt, n, inc, static_cast<float *>(dst));
    else host_convert(src, dt, n, inc, static_cast<int64_t *>(dst));
}

// Contiguous compute-eltype vector (F64 / F32 / I64) stored into a strided host vector of eltype
// `dt` (the compute eltype, or I32 from I64: Julia's wrapping truncation).
inline void host_store(const void *src, int cdt, int64_t n, void *dst, int dt, int64_t inc)
{
    char *p = static_cast<char *>(dst);
    const int esz = elem_size(dt);
    for (int64_t i = 0; i < n; i++) {
        char *e = p + i * inc * esz;
        if (dt == VBC_F64) *reinterpret_cast<double *>(e) = static_cast<const double *>(src)[i];
        else if (dt == VBC_F32) *reinterpret_cast<float *>(e) = static_cast<const float *>(src)[i];
        else if (dt == VBC_I64) *reinterpret_cast<int64_t *>(e) = static_cast<const int64_t *>(src)[i];
        else *reinterpret_cast<int32_t *>(e) = (int32_t) static_cast<const int64_t *>(src)[i];
    }
    (void)cdt;
}

}  // namespace vbc
