// FETCH_SIZE calibration on gfx950: read a known byte count (1 GiB, far past
// the 256 MiB Infinity Cache) at several per-lane access widths, so the PMC
// factor for this repo's access patterns is measured rather than assumed
// (MI355X_MICROARCH.md §HBM: FETCH_SIZE is calibrated only for 16 B/lane).
//   hipcc -O3 --offload-arch=gfx950 tools/calib_fetch.hip -o tools/build/calib_fetch
//   rocprofv3 --pmc FETCH_SIZE -d DIR -o run --output-format csv -- tools/build/calib_fetch
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <class T>
__global__ void read_width(const T* __restrict__ p, size_t n, unsigned* out) {
    unsigned acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        if constexpr (sizeof(T) == 16) {
            uint4 v = reinterpret_cast<const uint4*>(p)[i];
            acc += v.x ^ v.y ^ v.z ^ v.w;
        } else {
            acc += (unsigned)p[i];
        }
    }
    if (acc == 0x12345678u) out[0] = acc;  // keep the loads alive
}

// 2-D window gather like the LK staging: each wave reads a 28x28 u8 window
// (one u16 pair per lane-pixel) at a pseudo-random position; windows disjoint.
__global__ void read_windows(const uint8_t* __restrict__ img, int pitch, int nwin_x, unsigned* out) {
    const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, lane = threadIdx.x & 63;
    const int wx = wave % nwin_x, wy = wave / nwin_x;
    const uint8_t* base = img + (size_t)wy * 32 * pitch + wx * 32;
    unsigned acc = 0;
    for (int k = lane; k < 28 * 28; k += 64) {
        const int r = k / 28, c = k - r * 28;
        acc += base[(size_t)r * pitch + c];
    }
    if (acc == 0x12345678u) out[0] = acc;
}

int main() {
    const size_t bytes = size_t(1) << 30;
    void* buf;
    unsigned* out;
    if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&out, 4) != hipSuccess) return 1;
    (void)hipMemset(buf, 1, bytes);
    const int grid = 256 * 8 * 4, block = 256;
    for (int rep = 0; rep < 2; rep++) {
        read_width<uint4><<<grid, block>>>((const uint4*)buf, bytes / 16, out);
        read_width<uint32_t><<<grid, block>>>((const uint32_t*)buf, bytes / 4, out);
        read_width<uint16_t><<<grid, block>>>((const uint16_t*)buf, bytes / 2, out);
        read_width<uint8_t><<<grid, block>>>((const uint8_t*)buf, bytes, out);
        // 32768 x 32768 u8 image, windows on a 32-px grid: 1024 x 1024 windows of 28x28
        read_windows<<<1024 * 1024 / 4, 256>>>((const uint8_t*)buf, 32768, 1024, out);
    }
    (void)hipDeviceSynchronize();
    printf("bytes per read_width launch: %zu; read_windows: %zu\n", bytes, (size_t)1024 * 1024 * 28 * 28);
    return 0;
}
