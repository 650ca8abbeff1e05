#include "../hymet_amd/csrc/mm_chain.hip"
#include <cstdio>
#include <cstdlib>
using namespace hymet::mm;
__global__ void k(const int *in, const double *ind, int *o_max, int *o_a, int *o_b, double *o_min, int *o_shr) {
    const int l = threadIdx.x;
    o_max[l] = scan_max(in[l]);
    int a = in[l] % 7 - 3, b = in[l] % 11;
    scan_maxplus(a, b);
    o_a[l] = a; o_b[l] = b;
    o_min[l] = scan_min_d(ind[l]);
    o_shr[l] = shr1(in[l], -5);
}
int main() {
    int h[64]; double hd[64];
    for (int i = 0; i < 64; i++) h[i] = rand() % 1000, hd[i] = (rand() % 1000) * 0.5;
    int *d, *om, *oa, *ob, *os; double *dd, *omin;
    hipMalloc(&d, 256); hipMalloc(&om, 256); hipMalloc(&oa, 256); hipMalloc(&ob, 256); hipMalloc(&os, 256);
    hipMalloc(&dd, 512); hipMalloc(&omin, 512);
    hipMemcpy(d, h, 256, hipMemcpyHostToDevice); hipMemcpy(dd, hd, 512, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, dd, om, oa, ob, omin, os);
    int rm[64], ra[64], rb[64], rs[64]; double rmin[64];
    hipMemcpy(rm, om, 256, hipMemcpyDeviceToHost); hipMemcpy(ra, oa, 256, hipMemcpyDeviceToHost);
    hipMemcpy(rb, ob, 256, hipMemcpyDeviceToHost); hipMemcpy(rs, os, 256, hipMemcpyDeviceToHost);
    hipMemcpy(rmin, omin, 512, hipMemcpyDeviceToHost);
    int bad = 0, mx = -1; double mn = 1e300; int A = 0, B = kNegInf;
    for (int l = 0; l < 64; l++) {
        mx = h[l] > mx ? h[l] : mx;
        mn = hd[l] < mn ? hd[l] : mn;
        int a = h[l] % 7 - 3, b = h[l] % 11;
        // compose (A,B) then (a,b)
        int nB = (B + a > b) ? B + a : b; int nA = A + a; A = nA; B = nB;
        int shr = l == 0 ? -5 : h[l - 1];
        if (rm[l] != mx) { bad++; if (bad < 5) printf("max lane %d got %d want %d\n", l, rm[l], mx); }
        if (rmin[l] != mn) { bad++; if (bad < 10) printf("min lane %d got %g want %g\n", l, rmin[l], mn); }
        if (ra[l] != A || rb[l] != (B < kNegInf/2 ? rb[l] : B)) { bad++; if (bad < 15) printf("mp lane %d got (%d,%d) want (%d,%d)\n", l, ra[l], rb[l], A, B); }
        if (rs[l] != shr) { bad++; if (bad < 20) printf("shr lane %d got %d want %d\n", l, rs[l], shr); }
    }
    printf("bad=%d\n", bad);
    return 0;
}
