// Host cost per launch of an empty kernel by three HIP launch paths (batches of 100 launches timed
// on the host without waiting for the device; median of 30 batches):
//   hipLaunchKernelGGL (runtime-registered kernel), hipModuleLaunchKernel with a kernelParams
//   array, hipModuleLaunchKernel with the HIP_LAUNCH_PARAM_BUFFER config (what fa_asm.cpp uses).
// The module is this file's own code object (hipModuleLoad of the offload bundle is not needed:
// hipGetFuncBySymbol gives the hipFunction_t of the registered kernel).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

struct Args {
    void *p[8];
    unsigned u[20];
};

__global__ void empty_kernel(Args a) {
    if (a.u[0] == 12345u && threadIdx.x == 1000) ((unsigned *)a.p[0])[0] = 1;
}

template <class F>
double host_us(F f) {
    std::vector<double> per;
    for (int r = 0; r < 30; ++r) {
        auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < 100; ++i) f();
        auto t1 = std::chrono::steady_clock::now();
        per.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count() / 100);
        hipDeviceSynchronize();
    }
    std::sort(per.begin(), per.end());
    return per[per.size() / 2];
}

int main() {
    hipStream_t s;
    hipStreamCreate(&s);
    Args a{};
    for (int i = 0; i < 50; ++i) hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(256), 0, s, a);
    hipDeviceSynchronize();
    hipFunction_t fn;
    if (hipGetFuncBySymbol(&fn, reinterpret_cast<const void *>(empty_kernel)) != hipSuccess) {
        printf("hipGetFuncBySymbol failed\n");
        return 1;
    }
    const double t_ggl = host_us([&] { hipLaunchKernelGGL(empty_kernel, dim3(8, 12, 8), dim3(256), 0, s, a); });
    void *params[] = {&a};
    const double t_params = host_us([&] { hipModuleLaunchKernel(fn, 8, 12, 8, 256, 1, 1, 0, s, params, nullptr); });
    size_t sz = sizeof(a);
    void *cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &a, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz, HIP_LAUNCH_PARAM_END};
    const double t_cfg = host_us([&] { hipModuleLaunchKernel(fn, 8, 12, 8, 256, 1, 1, 0, s, nullptr, cfg); });
    const double t_err = host_us([&] { (void)hipGetLastError(); });
    int dev;
    const double t_dev = host_us([&] { (void)hipGetDevice(&dev); });
    printf("{\"hipLaunchKernelGGL_us\": %.3f, \"hipModuleLaunchKernel_params_us\": %.3f, "
           "\"hipModuleLaunchKernel_config_us\": %.3f, \"hipGetLastError_us\": %.3f, \"hipGetDevice_us\": %.3f}\n",
           t_ggl, t_params, t_cfg, t_err, t_dev);
    hipDeviceSynchronize();
    return 0;
}
