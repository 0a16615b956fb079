// Raw buffer loads/stores bound to the LLVM intrinsics by name. In this toolchain the clang
// builtins __builtin_amdgcn_raw_buffer_load_b64 / _b128 lower to a single buffer_load_dword
// (upper dwords undefined), so the wide forms are declared here instead.
#pragma once
#include <hip/hip_runtime.h>

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

extern "C" __device__ float rbuf_ld1(__amdgpu_buffer_rsrc_t, int, int, int) __asm("llvm.amdgcn.raw.ptr.buffer.load.f32");
extern "C" __device__ f32x2 rbuf_ld2(__amdgpu_buffer_rsrc_t, int, int, int) __asm("llvm.amdgcn.raw.ptr.buffer.load.v2f32");
extern "C" __device__ f32x4 rbuf_ld4(__amdgpu_buffer_rsrc_t, int, int, int) __asm("llvm.amdgcn.raw.ptr.buffer.load.v4f32");
extern "C" __device__ void rbuf_st1(float, __amdgpu_buffer_rsrc_t, int, int, int) __asm("llvm.amdgcn.raw.ptr.buffer.store.f32");
extern "C" __device__ void rbuf_st2(f32x2, __amdgpu_buffer_rsrc_t, int, int, int) __asm("llvm.amdgcn.raw.ptr.buffer.store.v2f32");
extern "C" __device__ void rbuf_st4(f32x4, __amdgpu_buffer_rsrc_t, int, int, int) __asm("llvm.amdgcn.raw.ptr.buffer.store.v4f32");
