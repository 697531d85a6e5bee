// capture_patterns.hip -- which multi-stream stream-capture patterns does
// HIP (ROCm 7.2) capture, instantiate and replay correctly?  One pattern per
// process (argv[1]), a trivial kernel per node; each kernel adds its node id
// into a per-node counter so the replay's execution can be checked.
//
//   0 fork/join  per iteration: record ev_fork on main, side waits it, side
//                kernel, record ev_side, main kernel, main waits ev_side --
//                every event waited on before it is recorded again (the
//                pattern of launch_step_rccl / launch_step_deferred)
//   1 banded     the removed banded pipeline (commit d83a934): B = 4 band
//                streams, events rotated mod 3 per band, each band waiting on
//                its neighbours' previous-iteration events and on every other
//                band's events two iterations back
//   2 banded-nr  pattern 1 without the two-iterations-back waits (redundant:
//                implied through the neighbours)
//   3 banded-1ev pattern 1 with one event per (iteration, band): no event is
//                recorded twice in the capture
//   4 rerecord   one event recorded twice on one stream before any wait, the
//                second record then waited on
//   5 fanout     one event recorded once, waited on by four streams, then
//                re-recorded and waited on again (the fork of pattern 1)
//   6 redundant  per iteration: A k, record e1; B waits e1, k, record e2; C
//                waits e2 and then e1 -- e1 is already an ancestor of C's
//                capture node when C waits on it
//   7 stale      per iteration: A k, record e1, k, record e1b; C waits e1 (no
//                longer A's last node, and not an ancestor of C's)
//   8 banded-b3  pattern 3 with B = 3 bands
//   9 banded-ord pattern 3 with the two-iterations-back waits issued before
//                the neighbour waits
//  10 banded-anc pattern 2 plus only the two-iterations-back waits on bands
//                at distance 2 (already ancestors through a neighbour)
//  11 banded-far pattern 2 plus only the two-iterations-back waits on bands
//                at distance >= 3 (not ancestors)
//
// usage: capture_patterns PATTERN ITERATIONS ; prints "pattern P n N: ok" or
// the failing call.  Build: hipcc --offload-arch=gfx950 -O2 -o
// scripts/micro/capture_patterns scripts/micro/capture_patterns.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                 \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) {                                                               \
            printf("pattern %d n %d: FAIL %s -> %s\n", pat, n, #x, hipGetErrorString(e_));    \
            return 1;                                                                         \
        }                                                                                     \
    } while (0)

__global__ void k_touch(unsigned *cnt, int node) { if (threadIdx.x == 0) atomicAdd(cnt + node, 1u); }

int main(int argc, char **argv)
{
    const int pat = argc > 1 ? atoi(argv[1]) : 0;
    const int n = argc > 2 ? atoi(argv[2]) : 50;
    constexpr int B = 4;
    hipStream_t main_s, st[B];
    CK(hipStreamCreateWithFlags(&main_s, hipStreamNonBlocking));
    for (auto &s : st) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    std::vector<hipEvent_t> ev((size_t)3 * B + (size_t)n * B + 4);
    for (auto &e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    unsigned *cnt;
    const int nodes = n * (B + 2) + 8;
    CK(hipMalloc(&cnt, sizeof(unsigned) * nodes));
    CK(hipMemset(cnt, 0, sizeof(unsigned) * nodes));
    CK(hipDeviceSynchronize());
    int node = 0;
    CK(hipStreamBeginCapture(main_s, hipStreamCaptureModeThreadLocal));
    if (pat == 0) {
        hipEvent_t fork = ev[0], side = ev[1];
        for (int j = 0; j < n; ++j) {
            CK(hipEventRecord(fork, main_s));
            CK(hipStreamWaitEvent(st[0], fork, 0));
            k_touch<<<1, 64, 0, st[0]>>>(cnt, node++);
            CK(hipEventRecord(side, st[0]));
            k_touch<<<1, 64, 0, main_s>>>(cnt, node++);
            CK(hipStreamWaitEvent(main_s, side, 0));
        }
    } else if ((pat >= 1 && pat <= 3) || (pat >= 8 && pat <= 11)) {
        hipEvent_t fork = ev[0];
        const int NB = pat == 8 ? 3 : B;
        const bool uniq = pat == 3 || pat >= 8;
        auto bev = [&](int j, int b) { return uniq ? ev[4 + (size_t)j * B + b] : ev[4 + (size_t)(j % 3) * B + b]; };
        auto back = [&](int j, int b) {  // the two-iterations-back waits
            if (j <= 1 || pat == 2) return;
            for (int b2 = 0; b2 < NB; ++b2) {
                const int d = b2 > b ? b2 - b : b - b2;
                if (d <= 1 || (pat == 10 && d != 2) || (pat == 11 && d < 3)) continue;
                if (hipStreamWaitEvent(st[b], bev(j - 2, b2), 0) != hipSuccess) { printf("wait failed\n"); exit(1); }
            }
        };
        k_touch<<<1, 64, 0, main_s>>>(cnt, node++);
        CK(hipEventRecord(fork, main_s));
        for (int b = 0; b < NB; ++b) CK(hipStreamWaitEvent(st[b], fork, 0));
        for (int j = 0; j < n; ++j) {
            for (int b = 0; b < NB; ++b) {
                if (pat == 9) back(j, b);
                if (j > 0) {
                    if (b > 0) CK(hipStreamWaitEvent(st[b], bev(j - 1, b - 1), 0));
                    if (b + 1 < NB) CK(hipStreamWaitEvent(st[b], bev(j - 1, b + 1), 0));
                }
                if (pat != 9) back(j, b);
                k_touch<<<1, 64, 0, st[b]>>>(cnt, node++);
                CK(hipEventRecord(bev(j, b), st[b]));
            }
        }
        for (int b = 0; b < NB; ++b) CK(hipStreamWaitEvent(main_s, bev(n - 1, b), 0));
    } else if (pat == 4) {
        hipEvent_t fork = ev[0], e = ev[1];
        for (int j = 0; j < n; ++j) {
            CK(hipEventRecord(fork, main_s));
            CK(hipStreamWaitEvent(st[0], fork, 0));
            k_touch<<<1, 64, 0, st[0]>>>(cnt, node++);
            CK(hipEventRecord(e, st[0]));
            k_touch<<<1, 64, 0, st[0]>>>(cnt, node++);
            CK(hipEventRecord(e, st[0]));  // re-recorded before anyone waited on it
            CK(hipStreamWaitEvent(main_s, e, 0));
        }
    } else if (pat == 5) {
        hipEvent_t fork = ev[0];
        for (int j = 0; j < n; ++j) {
            CK(hipEventRecord(fork, main_s));
            for (int b = 0; b < B; ++b) {
                CK(hipStreamWaitEvent(st[b], fork, 0));
                k_touch<<<1, 64, 0, st[b]>>>(cnt, node++);
                CK(hipEventRecord(ev[1 + b], st[b]));
            }
            for (int b = 0; b < B; ++b) CK(hipStreamWaitEvent(main_s, ev[1 + b], 0));
        }
    } else if (pat == 6 || pat == 7) {
        hipEvent_t fork = ev[0], e1 = ev[1], e2 = ev[2], e1b = ev[3], ej = ev[4];
        for (int j = 0; j < n; ++j) {
            CK(hipEventRecord(fork, main_s));
            for (int b = 0; b < 3; ++b) CK(hipStreamWaitEvent(st[b], fork, 0));
            k_touch<<<1, 64, 0, st[0]>>>(cnt, node++);
            CK(hipEventRecord(e1, st[0]));
            if (pat == 6) {
                CK(hipStreamWaitEvent(st[1], e1, 0));
                k_touch<<<1, 64, 0, st[1]>>>(cnt, node++);
                CK(hipEventRecord(e2, st[1]));
                CK(hipStreamWaitEvent(st[2], e2, 0));
                CK(hipStreamWaitEvent(st[2], e1, 0));  // redundant: e1 precedes e2
            } else {
                k_touch<<<1, 64, 0, st[0]>>>(cnt, node++);
                CK(hipEventRecord(e1b, st[0]));
                CK(hipStreamWaitEvent(st[2], e1, 0));  // not A's last node
                CK(hipStreamWaitEvent(main_s, e1b, 0));
            }
            k_touch<<<1, 64, 0, st[2]>>>(cnt, node++);
            CK(hipEventRecord(ej, st[2]));
            CK(hipStreamWaitEvent(main_s, ej, 0));
            if (pat == 6) CK(hipStreamWaitEvent(main_s, e2, 0));
        }
    }
    fprintf(stderr, "pattern %d n %d: calls issued\n", pat, n);
    hipGraph_t g;
    CK(hipStreamEndCapture(main_s, &g));
    fprintf(stderr, "pattern %d n %d: capture ended\n", pat, n);
    hipGraphExec_t ge;
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    fprintf(stderr, "pattern %d n %d: instantiated\n", pat, n);
    for (int rep = 0; rep < 3; ++rep) CK(hipGraphLaunch(ge, main_s));
    CK(hipStreamSynchronize(main_s));
    std::vector<unsigned> h(nodes);
    CK(hipMemcpy(h.data(), cnt, sizeof(unsigned) * nodes, hipMemcpyDeviceToHost));
    int bad = 0;
    for (int i = 0; i < node; ++i) bad += h[i] != 3u;
    printf("pattern %d n %d: %s (%d nodes, %d with a wrong count)\n", pat, n, bad ? "WRONG" : "ok", node, bad);
    return bad ? 2 : 0;
}
