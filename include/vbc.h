/*
 * vbc.h -- C ABI of libvbc, the MI355X-native variable-block SpMV library.
 *
 * Drop-in boundary for SparseMatrixVBCs.jl's hot path (reference @ /root/reference, v0.1.12).
 * Every entry point is what a Julia `ccall` shim would bind underneath the reference's own operator
 * surface (see INTEGRATION.md for the binding).  Plain pointers and sizes only: no torch types,
 * no C++ types.  All functions return an int status (vbc_status) and never throw.
 *
 * Index conventions at the boundary follow the Julia struct fields verbatim: 1-based Int64
 * (`Ti = Int64`) arrays, exactly as SparseMatrix1DVBC{W,Tv,Ti} / SparseMatrixVBC{U,W,Tv,Ti} /
 * SplitPartition{Ti} store them (SparseMatrixVBCs.jl:36-53, :62-82).  The library validates them and
 * converts once, at create time, into its own 0-based int32 HBM layout.
 */
#ifndef VBC_H
#define VBC_H

#ifndef VBC_API
#define VBC_API __attribute__((visibility("default")))  /* the library builds with -fvisibility=hidden */
#endif

#include <stddef.h>
#include <stdint.h>

/* ABI version (major*10000 + minor*100 + patch), returned by vbc_version().  A binding checks the major
 * version at load time: 3.x changed vbc_info (VBC_INFO_SIZE bytes, written whole by vbc_get_info) and
 * added the I64 / I32 / BOOL eltypes, the sharded 2D handle and the *_ex sharded product. */
#define VBC_VERSION 30200
#define VBC_INFO_SIZE 152

#ifdef __cplusplus
extern "C" {
#endif

/* Status codes.  The Julia shim maps them onto the reference's exceptions:
 * DimensionMismatch (multiply_1DVBC.jl:44-45,139-140), ArgumentError (SparseMatrixVBCs.jl:45-50,
 * :72-79) and AssertionError (constructors_1DVBC.jl:46, constructors_VBC.jl:59,65). */
typedef enum vbc_status {
    VBC_OK = 0,
    VBC_DIM_MISMATCH = 1,      /* -> DimensionMismatch() */
    VBC_INVALID_ARG = 2,       /* -> ArgumentError(msg) */
    VBC_HIP_ERROR = 3,         /* -> ErrorException(msg) */
    VBC_RCCL_ERROR = 4,        /* -> ErrorException(msg) */
    VBC_UNSUPPORTED_DTYPE = 5, /* -> MethodError-like: no GPU kernel for this eltype */
    VBC_ASSERTION = 6          /* -> AssertionError (w <= W, u <= U) */
} vbc_status;

/* Element types.  vbc*_create / vbc_mul / vbc_mul_mat: Tv = x = y = F64 or F32.  The *_ex entry
 * points below add the reference's other eltypes (Bool and Int32 matrices: runtests.jl:15-16; the
 * product computes in eltype(y): multiply_1DVBC.jl:27,34,102) and Int32 index arrays (Ti). */
typedef enum vbc_dtype {
    VBC_F64 = 0,
    VBC_F32 = 1,
    VBC_I64 = 2,  /* Int64: exact two's-complement wrapping arithmetic (Julia Int64 semantics)     */
    VBC_I32 = 3,  /* Int32: computed as Int64, stored back truncated (Julia Int32 wraparound)      */
    VBC_BOOL = 4  /* Bool as one byte, 0 / 1 (values and x only)                                     */
} vbc_dtype;

/* Where x / y live for vbc_mul / vbc_mul_mat. */
typedef enum vbc_mem { VBC_MEM_DEVICE = 0, VBC_MEM_HOST = 1 } vbc_mem;

/* create flags */
#define VBC_CREATE_TRANSPOSED 0x1u /* build the layout for mul!(y, B', x)  (default if 0 given) */
#define VBC_CREATE_FORWARD 0x2u    /* build the layout for mul!(y, B, x)                         */
#define VBC_CREATE_MULTI 0x4u      /* build the panel layout of the multi-RHS transposed product
                                      Y = α·B'X + β·Y on matrix cores (vbc_mul_mat, trans = 1,
                                      any operand layout; stripes wider than 16 are cut into
                                      16-column pieces).  Independent of the SpMV layouts. */
#define VBC_CREATE_MULTI_FORWARD 0x10u /* build the panel layout of the multi-RHS FORWARD product
                                      Y = α·B·X + β·Y on matrix cores (vbc_mul_mat, trans = 0): the
                                      panel layout of Bᵀ -- output row groups (Π's block rows of a
                                      SparseMatrixVBC; runs of rows with identical stripe lists of a
                                      1DVBC, <= 16) as stripes, every tile column a stored row -- so the
                                      matrix is read once for all right-hand sides. */
#define VBC_CREATE_SERIAL 0x8u     /* keep the reference's serial summation order in every layout of
                                      both directions: no split planar B'x product (per-stripe row
                                      order, multiply_1DVBC.jl:101-104; vbc_info.planar_split stays 1),
                                      no merge layout where a slotted one can hold the bucket (its
                                      segmented scan joins per-slot partial sums), and no split
                                      forward product (stripe order per output row, :62-71; planar_mask
                                      bit 3 stays clear), so every B'x output is bit-identical to the
                                      oracle whatever the matrix size (B·x: see VBC_SPLIT_ROWS).  Default:
                                      small matrices may fold a chunk's rows (B'x) or blocks (B·x) in
                                      P slices whose partial sums meet in LDS (rounding differs ~1 ulp);
                                      vbc_info reports it as planar_split > 1 / planar_mask bit 3. */

/* mul flags */
#define VBC_MAT_ROWMAJOR 0x2u         /* vbc_mul_mat: X, Y row-major (right-hand sides interleaved,
                                         X[i*ldx + j], ld >= nrhs); the fused multi-RHS kernel
                                         reads one contiguous X row per stored row.  Default:
                                         column-major (Julia), one SpMV per column. */
#define VBC_MUL_REFERENCE_QUIRKS 0x1u /* reproduce the reference bit-for-bit in alpha/beta:
                                         forward drops alpha (multiply_1DVBC.jl:48,
                                         multiply_VBC.jl:55-57); transposed overwrites y, ignoring
                                         alpha and beta (multiply_1DVBC.jl:114-116,
                                         multiply_VBC.jl:117-121).  Default (0) is BLAS:
                                         y = alpha*op(B)*x + beta*y.  Both agree at (1, 0). */

typedef struct vbc_handle vbc_handle; /* opaque; immutable after create */

/* ---------------------------------------------------------------------------------------------
 * Handles (device-resident matrices)
 * ------------------------------------------------------------------------------------------- */

/* SparseMatrix1DVBC{W,Tv,Int64}(m, n, Φ, pos, idx, ofs, val)  (SparseMatrixVBCs.jl:36-53).
 * spl[L+1] = Φ.spl, pos[L+1], idx[pos[L+1]-1], ofs[L+1]: 1-based Int64.  val has nval >=
 * ofs[L+1]-1 elements (the reference's SIMD tail pad, constructors_1DVBC.jl:35-39, is ignored).
 * `device` is the HIP ordinal; `flags` selects which product layouts to build (0 = transposed). */
VBC_API int vbc1d_create(vbc_handle **out, int64_t m, int64_t n, int64_t W, int64_t L, const int64_t *spl,
                 const int64_t *pos, const int64_t *idx, const int64_t *ofs, const void *val,
                 int64_t nval, int dtype, int device, unsigned flags);

/* SparseMatrixVBC{U,W,Tv,Int64}(m, n, Π, Φ, pos, idx, ofs, val)  (SparseMatrixVBCs.jl:62-82).
 * pspl[K+1] = Π.spl; idx holds block-row ids k (constructors_VBC.jl:123). */
VBC_API int vbc2d_create(vbc_handle **out, int64_t m, int64_t n, int64_t U, int64_t W, int64_t K,
                 const int64_t *pspl, int64_t L, const int64_t *spl, const int64_t *pos,
                 const int64_t *idx, const int64_t *ofs, const void *val, int64_t nval, int dtype,
                 int device, unsigned flags);

/* SparseMatrixCSC{Tv,Int64} (colptr[n+1], rowval, nzval), the operand of TrSpMV!(y, A, x)
 * (TrSpMV.jl:1-20).  Internally a 1DVBC with unit-width stripes. */
VBC_API int vbc_csc_create(vbc_handle **out, int64_t m, int64_t n, const int64_t *colptr,
                   const int64_t *rowval, const void *nzval, int dtype, int device, unsigned flags);

VBC_API int vbc_destroy(vbc_handle *h);

/* Type parameters of the *_ex create calls: the reference's SparseMatrix1DVBC{W,Tv,Ti} with any
 * Tv in {Float64, Float32, Int64, Int32, Bool} and Ti in {Int64, Int32}, and the eltype the products
 * compute in.  The reference computes in eltype(y) (multiply_1DVBC.jl:27,34,102 convert val and x to
 * it), so a binding creates one handle per eltype(y) it meets:
 *   compute_dtype = VBC_F64 / VBC_F32: values converted once at create (Bool / integer -> float is
 *                   exact below 2^53 / 2^24); the float kernels (slotted / swept / merge / panel);
 *   compute_dtype = VBC_I64: Int64 values, exact wrapping arithmetic (vbc_generic.hip), for
 *                   integer y (Int64, or Int32 stored back truncated -- Julia's wraparound). */
typedef struct vbc_types {
    int32_t val_dtype;     /* eltype of val / nzval as passed (vbc_dtype) */
    int32_t index_bits;    /* 64 or 32: width of spl / pos / idx / ofs (colptr / rowval, Π.spl) */
    int32_t compute_dtype; /* VBC_F64, VBC_F32 or VBC_I64 */
    int32_t reserved;      /* 0 */
} vbc_types;

VBC_API int vbc1d_create_ex(vbc_handle **out, int64_t m, int64_t n, int64_t W, int64_t L, const void *spl,
                            const void *pos, const void *idx, const void *ofs, const void *val, int64_t nval,
                            const vbc_types *types, int device, unsigned flags);
VBC_API int vbc2d_create_ex(vbc_handle **out, int64_t m, int64_t n, int64_t U, int64_t W, int64_t K,
                            const void *pspl, int64_t L, const void *spl, const void *pos, const void *idx,
                            const void *ofs, const void *val, int64_t nval, const vbc_types *types, int device,
                            unsigned flags);
VBC_API int vbc_csc_create_ex(vbc_handle **out, int64_t m, int64_t n, const void *colptr, const void *rowval,
                              const void *nzval, const vbc_types *types, int device, unsigned flags);

/* ---------------------------------------------------------------------------------------------
 * Products
 * ------------------------------------------------------------------------------------------- */

/* mul!(y, B, x, α, β) (trans = 0; multiply_1DVBC.jl:9-83, multiply_VBC.jl:3-87) or
 * mul!(y, B', x, α, β) (trans = 1; multiply_1DVBC.jl:85-180, multiply_VBC.jl:89-192, and
 * TrSpMV!(y, A, x) for a CSC handle, TrSpMV.jl:1-20).  Adjoint and Transpose are identical (real
 * eltypes only).  nx / ny are length(x) / length(y): a mismatch returns VBC_DIM_MISMATCH before any
 * work.  mem = VBC_MEM_DEVICE: x, y are device pointers on the handle's device, and the product is
 * enqueued on `stream` (a hipStream_t; NULL = null stream) without synchronising.  A transposed
 * product whose buckets need several independent launches may run some of them on side streams the
 * handle owns: they wait for an event recorded on `stream` and are joined back into it before the call
 * returns, so every later operation on `stream` (and a HIP graph captured from it) sees the whole y.
 * mem = VBC_MEM_HOST: x, y are host pointers; the call stages them and returns when y is final.
 * x and y must not alias (the reference has the same precondition).  x and y are contiguous vectors of
 * the handle's compute eltype: this is the fast path for callers that know it (the Python mirror after
 * its own eltype check); a binding that cannot guarantee it calls vbc_mul_ex, which carries them. */
VBC_API int vbc_mul(vbc_handle *h, int trans, const void *x, int64_t nx, void *y, int64_t ny, double alpha,
            double beta, int mem, void *stream, unsigned flags);

/* mul!(y::StridedVector, op(B), x::StridedVector, α, β) with any strides and eltypes the
 * reference accepts (multiply_1DVBC.jl:9,85 take StridedVector; :102 converts x to eltype(y)).
 * x_dtype: any vbc_dtype, converted to the handle's compute eltype (a float x is refused on an
 * integer handle: Julia's convert would throw InexactError); y_dtype: the compute eltype, or VBC_I32
 * on an integer handle.  incx / incy: element strides (any nonzero value; negative = reversed view,
 * the pointer is that of x[1] / y[1]).  Contiguous operands of the compute eltype go straight to the
 * kernels; others through the handle's staging buffers (a conversion kernel on each side).
 * mem, stream, flags as vbc_mul. */
VBC_API int vbc_mul_ex(vbc_handle *h, int trans, const void *x, int x_dtype, int64_t incx, int64_t nx, void *y,
                       int y_dtype, int64_t incy, int64_t ny, double alpha, double beta, int mem, void *stream,
                       unsigned flags);

/* Multi-RHS Y = α·op(B)·X + β·Y.  X is nx × nrhs, Y is ny × nrhs; column-major (ldx >= nx, ldy >=
 * ny) by default, row-major with VBC_MAT_ROWMAJOR (ldx, ldy >= nrhs).  The reference has no matrix
 * mul! (Base.:* forwards to an undefined method, multiply_1DVBC.jl:184-185), so the semantics is
 * defined column by column as vbc_mul.  trans = 1 on a handle with VBC_CREATE_MULTI: one
 * matrix-core pass per 64 right-hand sides, row- or column-major.  Otherwise the transposed
 * row-major product with widths <= 8 runs a fused vector kernel over the SpMV layout, and the other
 * cases run one SpMV per column. */
VBC_API int vbc_mul_mat(vbc_handle *h, int trans, int64_t nrhs, const void *X, int64_t ldx, int64_t nx,
                void *Y, int64_t ldy, int64_t ny, double alpha, double beta, int mem, void *stream,
                unsigned flags);

/* vbc_mul_mat with the eltypes of X and Y carried along: both must be the handle's compute eltype
 * (VBC_UNSUPPORTED_DTYPE otherwise -- never read as another type); a binding with other eltypes runs
 * vbc_mul_ex column by column, as the reference's per-column semantics allows. */
VBC_API int vbc_mul_mat_ex(vbc_handle *h, int trans, int64_t nrhs, const void *X, int X_dtype, int64_t ldx,
                           int64_t nx, void *Y, int Y_dtype, int64_t ldy, int64_t ny, double alpha, double beta,
                           int mem, void *stream, unsigned flags);

/* ---------------------------------------------------------------------------------------------
 * Multi-GPU (one process, several GPUs of a node; RCCL over xGMI).  SURVEY.md §8e.
 *
 * Replaces the reference's only parallel region, the threaded stripe loop of the transposed product
 * (multiply_1DVBC.jl:169-177, multiply_VBC.jl:182-189), by a split of the matrix over GPUs: ranges
 * balanced by HBM bytes, one single-GPU handle per device (vbc1d_create_ex on each slice).
 *   VBC_SPLIT_STRIPES: GPU g owns stripes [l_g, l_g+1) (columns [c_g, c_g+1) of B; block rows of A
 *     when B stores Aᵀ, as bin/test_table.jl:27 does).  B'x: each GPU receives the span of x its stripes
 *     read (vbc_sharded_xspan; a mesh operator's shard: its share plus a halo), y slices gathered to the
 *     root (disjoint; each stripe summed in stored row order, bit-identical to one GPU and to the
 *     reference, unless a shard's layout runs the split planar product -- vbc_info.planar_split > 1,
 *     small shards only -- which sums a chunk's rows in P slices; VBC_CREATE_SERIAL forbids it).
 *     The disjoint B·x slices of VBC_SPLIT_ROWS keep each output row's stripe order
 *     (multiply_1DVBC.jl:62-71) but a shard may run another forward kernel family than the whole
 *     matrix (vbc_info fwd_run / planar_mask bits 1, 3, 4 / slot_bins): the slotted and planar forward
 *     kernels associate a block's w-term dot product differently (~1 ulp), and a small shard may run
 *     the split forward product (planar_mask bit 3), which VBC_CREATE_SERIAL forbids.
 *     Bx: x slices scattered, ncclReduce(sum) of y.
 *   VBC_SPLIT_ROWS: GPU g owns the stored rows [r_g, r_g+1) of every stripe.  Bx: the span of x its
 *     stripes read (vbc_sharded_xspan) to each GPU, y slices gathered (disjoint).  B'x: x slices, ncclReduce(sum) of y.
 * devices: all distinct (one RCCL communicator per device, ncclCommInitAll) or all the same device
 * (shards share it; no communicators -- oversubscription and single-GPU testing).
 * ------------------------------------------------------------------------------------------- */
typedef struct vbc_sharded vbc_sharded; /* opaque */
#define VBC_SPLIT_STRIPES 0
#define VBC_SPLIT_ROWS 1
/* VBC_SPLIT_AUTO: the split with the smaller predicted time of the products `flags` builds (B'x when
 * VBC_CREATE_TRANSPOSED or no direction flag is given, B x when VBC_CREATE_FORWARD): per product the slowest
 * shard's kernel (3.1 us + its bytes at 5.7 TB/s, both measured on one MI355X) plus the exchange through
 * devices[0] (x spans over the root's links + y slices gathered, or x slices + ncclReduce of y) at ASSUMED
 * xGMI rates of 76.8 GB/s x 0.6 per link, 7 links, 2 us per ring step; costs within 2 % tie, and a
 * tie goes to the split with disjoint outputs for the one direction built (stripes when both are built).
 * vbc_sharded_split reports the choice. */
#define VBC_SPLIT_AUTO 2

/* Same matrix arguments as vbc1d_create_ex (types: Tv, Ti, compute eltype); `flags` as vbc1d_create
 * (the layouts each shard builds). */
VBC_API int vbc1d_create_sharded(vbc_sharded **out, int64_t m, int64_t n, int64_t W, int64_t L, const void *spl,
                                 const void *pos, const void *idx, const void *ofs, const void *val, int64_t nval,
                                 const vbc_types *types, int ngpus, const int *devices, int split, unsigned flags);

/* SparseMatrixVBC{U,W,Tv,Ti} split the same way (its transposed product is threaded like the 1D one,
 * multiply_VBC.jl:182-189).  Same matrix arguments as vbc2d_create_ex.
 *   VBC_SPLIT_STRIPES: GPU g owns stripes [l_g, l_g+1) (Π kept whole);
 *   VBC_SPLIT_ROWS:    GPU g owns the block rows [k_g, k_g+1) of Π (rows Π.spl[k_g]-1 ..), i.e. the
 *                      tiles of every stripe whose block-row id falls in that range, stored order kept. */
VBC_API int vbc2d_create_sharded(vbc_sharded **out, int64_t m, int64_t n, int64_t U, int64_t W, int64_t K,
                                 const void *pspl, int64_t L, const void *spl, const void *pos, const void *idx,
                                 const void *ofs, const void *val, int64_t nval, const vbc_types *types, int ngpus,
                                 const int *devices, int split, unsigned flags);

/* mul!(y, op(B), x, α, β) over all shards, operands of the compute eltype: the fast path for a caller
 * that already holds contiguous x, y of that eltype (a binding that cannot guarantee it calls
 * vbc_sharded_mul_ex, which carries the eltypes).  mem = VBC_MEM_DEVICE: x, y live on devices[0] and the
 * product -- collectives included -- is ordered on `stream` (a hipStream_t of devices[0]) without host
 * synchronisation.  mem = VBC_MEM_HOST: host x, y; returns when y is final.  Products of one sharded
 * handle are issued one at a time (an internal lock keeps every GPU's collective order identical).
 * A failure after the first collective of a product was enqueued leaves the handle FAILED: the
 * communicators may hold a half-issued exchange, so every later product returns VBC_RCCL_ERROR
 * (destroy and re-create the handle). */
VBC_API int vbc_sharded_mul(vbc_sharded *s, int trans, const void *x, int64_t nx, void *y, int64_t ny, double alpha,
                            double beta, int mem, void *stream, unsigned flags);

/* mul!(y::StridedVector, op(B), x::StridedVector, α, β) on a sharded handle: eltypes and strides as
 * vbc_mul_ex (x converted to the compute eltype, multiply_1DVBC.jl:9,85,102; y the compute eltype or
 * Int32 on an integer handle; a mismatched eltype is converted or refused, never read as another
 * type).  Non-contiguous or converted operands go through root staging buffers (device) or host copies. */
VBC_API int vbc_sharded_mul_ex(vbc_sharded *s, int trans, const void *x, int x_dtype, int64_t incx, int64_t nx,
                               void *y, int y_dtype, int64_t incy, int64_t ny, double alpha, double beta, int mem,
                               void *stream, unsigned flags);

VBC_API int vbc_sharded_destroy(vbc_sharded *s);
VBC_API int vbc_sharded_count(const vbc_sharded *s, int *ngpus);
/* The split the handle uses (VBC_SPLIT_STRIPES or VBC_SPLIT_ROWS; what VBC_SPLIT_AUTO chose). */
VBC_API int vbc_sharded_split(const vbc_sharded *s, int *split);
/* Shard g: its single-GPU handle (owned by s), its 0-based range [lo, hi) of the split dimension
 * (columns for VBC_SPLIT_STRIPES, rows for VBC_SPLIT_ROWS) and its device. */
VBC_API int vbc_sharded_shard(const vbc_sharded *s, int g, vbc_handle **h, int64_t *lo, int64_t *hi, int *device);
/* Shard g's x span: the 0-based range [lo, hi) of x that its disjoint-output product reads (the rows its
 * stripes store for VBC_SPLIT_STRIPES' B'x, the columns of the stripes with a stored row in its range for
 * VBC_SPLIT_ROWS' B x; [0, 0) when it reads none).  devices[0] sends each shard that span instead of
 * broadcasting x; a caller that distributes x itself needs no more on shard g's device. */
VBC_API int vbc_sharded_xspan(const vbc_sharded *s, int g, int64_t *lo, int64_t *hi);

/* ---------------------------------------------------------------------------------------------
 * Introspection (for the Julia shim's size(), and for roofline accounting in bench.py)
 * ------------------------------------------------------------------------------------------- */
typedef struct vbc_info {
    int64_t m, n;          /* size(A) */
    int64_t L;             /* stripes */
    int64_t K;             /* block rows (2D), 0 for 1D */
    int64_t nblocks;       /* stored row-blocks q (2D: stored u×w tiles) */
    int64_t nrows;         /* stored w-wide rows after 2D expansion (== nblocks for 1D) */
    int64_t nval;          /* |val| = ofs[L+1]-1 (includes fill zeros) */
    int64_t nnz_hint;      /* nonzeros of val (useful flops = 2*nnz_hint) */
    int32_t dtype;
    int32_t device;
    int32_t bins_t, bins_f; /* kernel bins built for each direction (0 = layout absent) */
    int64_t device_bytes;   /* HBM held by the handle */
    int64_t bytes_t;        /* HBM bytes one transposed product moves in this layout */
    int64_t bytes_f;        /* same for the forward product */
    int32_t bins_m;         /* width buckets of the multi-RHS panel layout (0 = absent; a handle built with
                               VBC_CREATE_MULTI_FORWARD only: those of its Bᵀ layout, bytes_m likewise) */
    int32_t slot_bins;      /* buckets laid out slotted (vbc_slots.h / vbc_planar.h), both directions */
    int64_t bytes_m;        /* matrix bytes (keys + values, panel-padded) one panel pass streams */
    int32_t sweep_bins;     /* B'x buckets laid out row-swept (vbc_sweep.hip) */
    int32_t planar_bins;    /* B'x buckets laid out planar (vbc_planar.h) */
    int32_t planar_run;     /* longest row run of those buckets (1 = none; 2, 3: one x gather per run) */
    int32_t planar_split;   /* waves per chunk of the split planar product (1 = one wave per range) */
    int32_t planar_pair;    /* 1: fp64 3-wide runs laid out for lane pairs (one 16-B gather per lane) */
    int32_t fwd_run;        /* forward product: output rows in runs of fwd_run share one x-slice gather */
    int32_t planar_mask;    /* bit 0: a B'x planar bucket, bit 1: the forward planar bucket, in masked chunk-local
                               length order (padding lanes fetch nothing); bit 2: a B'x planar bucket in
                               per-lane compacted streams (tiles of stripes dealt to the lanes); bit 3:
                               the forward product sums some chunk's blocks in P slices (a split forward
                               planar bucket, or -- with bit 8 -- a split bin of C = Bᵀ's layout);
                               bit 4: the forward bucket in lane streams (node blocks transposed);
                               bit 5: a small matrix's B'x buckets of every width (1..8) laid out planar
                               and split, run by ONE fused launch (planar_split = its P); bit 6: some of
                               those stripes cut into 2 / 4 lane parts (long stripes); bit 7: reserved (0;
                               round 5's VALU stripe-quad layout); bit 8: the
                               forward product runs on the transposed layout of C = Bᵀ (stripes of several
                               widths: one fused launch instead of one per width); bit 9: the multi-RHS
                               layout has tile-granular buckets (u, w <= 4 tiles: one key and one u-row X
                               block per tile, spmm_tiles); bit 10: reserved (0; round 5's staged-X tile
                               form); bit 11: the forward product of 3 x 3 fp64 node blocks in the lane-pair
                               layout of the transposed blocks (spmv_planar_pair DOT, round 6) */
} vbc_info;

/* Writes VBC_INFO_SIZE bytes: `info` must be a vbc_info of this header's version (vbc_version() /
 * 10000 == VBC_VERSION / 10000). */
VBC_API int vbc_get_info(const vbc_handle *h, vbc_info *info);

/* Copies the thread's last error message (NUL-terminated, truncated to n). Returns its length. */
VBC_API int vbc_last_error(char *buf, size_t n);

/* Library version (major*10000 + minor*100 + patch). */
VBC_API int vbc_version(void);

#ifdef __cplusplus
}
#endif
#endif /* VBC_H */
