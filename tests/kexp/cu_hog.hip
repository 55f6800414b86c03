// CU hog (test tooling, not product): K workgroups that each hold a CU's worth of LDS and
// spin for a fixed wall time, launched on a side stream beside a training step -- what the
// RCCL all-reduce kernels of a data-parallel step do to the persistent one-workgroup-per-CU
// kernels (stem, big-box conv, ConvTranspose stream) while a gradient bucket is in flight.
// Built by tests/kexp/Makefile (libcuhog.so), driven by tests/kexp/cu_hog.py.
//
// hog_kernel: 64 threads, 2 VGPRs and (the compiler drops the never-written array) no LDS:
// it blocks only kernels that fill a SIMD's register file.  rccl_like_kernel: the footprint of
// RCCL's ncclDevKernel_Generic on gfx950 (librccl.so code-object metadata: 37,664 B of LDS,
// 248-256 VGPRs, 256-512 threads per workgroup) -- 256 threads, the LDS written so it stays
// allocated, 248 VGPRs forced by an asm clobber.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {
__global__ void __launch_bounds__(64) hog_kernel(unsigned long long ticks, int* sink) {
  __shared__ int pad[6144];
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();  // 100 MHz
  int v = 0;
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) {
    __builtin_amdgcn_s_sleep(8);
    v += pad[(threadIdx.x + v) & 63];
  }
  if (v == 0x7fffffff) sink[threadIdx.x] = v;  // keeps the loop (never true: pad is never written)
}

constexpr int kRcclLdsInts = 37664 / 4;
__global__ void __launch_bounds__(256) rccl_like_kernel(unsigned long long ticks, int* sink) {
  __shared__ int pad[kRcclLdsInts];
  for (int i = threadIdx.x; i < kRcclLdsInts; i += 256) pad[i] = i;
  __syncthreads();
  asm volatile("" ::: "v0", "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v8", "v9", "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "v18", "v19", "v20", "v21", "v22", "v23", "v24", "v25", "v26", "v27", "v28", "v29", "v30", "v31", "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "v64", "v65", "v66", "v67", "v68", "v69", "v70", "v71", "v72", "v73", "v74", "v75", "v76", "v77", "v78", "v79", "v80", "v81", "v82", "v83", "v84", "v85", "v86", "v87", "v88", "v89", "v90", "v91", "v92", "v93", "v94", "v95", "v96", "v97", "v98", "v99", "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107", "v108", "v109", "v110", "v111", "v112", "v113", "v114", "v115", "v116", "v117", "v118", "v119", "v120", "v121", "v122", "v123", "v124", "v125", "v126", "v127", "v128", "v129", "v130", "v131", "v132", "v133", "v134", "v135", "v136", "v137", "v138", "v139", "v140", "v141", "v142", "v143", "v144", "v145", "v146", "v147", "v148", "v149", "v150", "v151", "v152", "v153", "v154", "v155", "v156", "v157", "v158", "v159", "v160", "v161", "v162", "v163", "v164", "v165", "v166", "v167", "v168", "v169", "v170", "v171", "v172", "v173", "v174", "v175", "v176", "v177", "v178", "v179", "v180", "v181", "v182", "v183", "v184", "v185", "v186", "v187", "v188", "v189", "v190", "v191", "v192", "v193", "v194", "v195", "v196", "v197", "v198", "v199", "v200", "v201", "v202", "v203", "v204", "v205", "v206", "v207", "v208", "v209", "v210", "v211", "v212", "v213", "v214", "v215", "v216", "v217", "v218", "v219", "v220", "v221", "v222", "v223", "v224", "v225", "v226", "v227", "v228", "v229", "v230", "v231", "v232", "v233", "v234", "v235", "v236", "v237", "v238", "v239", "v240", "v241", "v242", "v243", "v244", "v245", "v246", "v247");
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  int v = 0;
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) {
    __builtin_amdgcn_s_sleep(8);
    v += pad[(threadIdx.x * 7 + v) % kRcclLdsInts];
  }
  if (v == 0x7fffffff) sink[threadIdx.x & 63] = v;
}
}  // namespace

// K workgroups spinning for us microseconds on stream s
extern "C" int cu_hog(int k, double us, int* sink, hipStream_t s) {
  if (k <= 0) return 0;
  hipLaunchKernelGGL(hog_kernel, dim3(k), dim3(64), 0, s, (unsigned long long)(us * 100.0), sink);
  return (int)hipGetLastError();
}

// K RCCL-footprint workgroups spinning for us microseconds on stream s
extern "C" int cu_hog_rccl(int k, double us, int* sink, hipStream_t s) {
  if (k <= 0) return 0;
  hipLaunchKernelGGL(rccl_like_kernel, dim3(k), dim3(256), 0, s, (unsigned long long)(us * 100.0), sink);
  return (int)hipGetLastError();
}
