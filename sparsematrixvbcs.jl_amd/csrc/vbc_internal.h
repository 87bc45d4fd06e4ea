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

inline int elem_size(int dtype) { return dtype == VBC_F64 ? 8 : dtype == VBC_F32 ? 4 : 0; }

}  // namespace vbc
