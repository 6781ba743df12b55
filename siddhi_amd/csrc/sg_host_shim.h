// Host-only compilation shim: lets tests/host_interp build the same __host__ __device__ machine code with
// g++ so its logic can be checked against the oracle without a GPU.  Never part of libsiddhi_gpu.so.
#pragma once
#include <cstring>
#include <cstdint>
#include <cmath>
#define __host__
#define __device__
#define __forceinline__ inline
#define SG_GLOBAL
static inline unsigned int __float_as_uint(float f) { unsigned int u; memcpy(&u, &f, 4); return u; }
static inline float __uint_as_float(unsigned int u) { float f; memcpy(&f, &u, 4); return f; }
static inline long long __double_as_longlong(double d) { long long u; memcpy(&u, &d, 8); return u; }
static inline double __longlong_as_double(long long u) { double d; memcpy(&d, &u, 8); return d; }
