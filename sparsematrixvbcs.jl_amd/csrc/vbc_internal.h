// Internal helpers shared by the host and device translation units of libvbc.
#pragma once
#include <cstdarg>
#include <cstdint>
#include <cstdio>

#include "vbc.h"

namespace vbc {

// Thread-local last-error message (vbc_last_error).
void set_error(const char *fmt, ...) __attribute__((format(printf, 1, 2)));

inline int fail(int status, const char *what)
{
    set_error("%s", what);
    return status;
}

inline int elem_size(int dtype)
{
    switch (dtype) {
    case VBC_F64: case VBC_I64: return 8;
    case VBC_F32: case VBC_I32: return 4;
    case VBC_BOOL: return 1;
    default: return 0;
    }
}

}  // namespace vbc
