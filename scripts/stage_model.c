/*
 * stage_model.c — CPU model: how much of the deferral
 * kernel's staged-sample traffic a hybrid resolve could avoid.
 *
 * With the tail rings on, every sample of a launch is staged (16 B) and
 * k_resolve_wave reduces them afterwards (16 B in per sample, 16 B out per
 * pixel): on C3 that is 265 MB written by the trace kernel and 299 MB moved
 * by the resolve per frame, 0.054 ms of resolve per 2.5 ms frame.  A hybrid
 * would resolve in the wave (the fused shuffle tree) every pixel of a chunk
 * whose 8 samples all finished in that wave, and stage only the pixels that
 * had a sample parked in the tail ring.  This replays the deferral rule
 * exactly on the oracle's per-path query counts (the same (pixel, sample,
 * frame) seeds as the GPU): a chunk is 64 consecutive paths (8 pixels x 8
 * spp); at the top of bounce n >= 1 the wave parks its live lanes once at
 * most DEFER (32) are live -- a lane is live at the top of bounce n iff its
 * path runs more than n queries; the ring reservation is assumed to succeed
 * (it retries at the next bounce when it does not, which parks fewer lanes).
 *
 * Build: gcc -O2 -fopenmp -ffp-contract=off -o /tmp/stage_model scripts/stage_model.c -lm
 * Run:   python scripts/dump_scene.py 32 /tmp/scene32.bin 1920 1080   (also writes /tmp/scene32.bin.uni)
 *        /tmp/stage_model /tmp/scene32.bin 1920 1080 8 8 8 [row_step] [frame] [defer]
 * Output: one JSON object (profiles/r05/stage_model_c3.json).
 */
#include "../oracle/mm_oracle.c"

#include <stdio.h>

static oracle_scene S;

static void load(const char* path) {
    FILE* f = fopen(path, "rb");
    if (!f) { perror(path); exit(1); }
    uint32_t nn[2];
    if (fread(nn, 4, 2, f) != 2) exit(1);
    S.n_rects = nn[0]; S.n_nodes = nn[1];
    mm_rect* r = malloc(sizeof(mm_rect) * S.n_rects);
    mm_node* n = malloc(sizeof(mm_node) * S.n_nodes);
    uint32_t* idx = malloc(4 * S.n_rects);
    uint8_t* m = malloc(S.n_rects);
    float* e = malloc(16 * S.n_rects);
    if (fread(r, sizeof(mm_rect), S.n_rects, f) != S.n_rects) exit(1);
    if (fread(n, sizeof(mm_node), S.n_nodes, f) != S.n_nodes) exit(1);
    if (fread(idx, 4, S.n_rects, f) != S.n_rects) exit(1);
    if (fread(m, 1, S.n_rects, f) != S.n_rects) exit(1);
    if (fread(e, 16, S.n_rects, f) != S.n_rects) exit(1);
    fclose(f);
    S.rects = r; S.nodes = n; S.idx = idx; S.is_mirror = m; S.emission = e;
}

int main(int argc, char** argv) {
    if (argc < 7) { fprintf(stderr, "usage: %s scene.bin W H spp bl ml [row_step] [frame] [defer]\n", argv[0]); return 2; }
    load(argv[1]);
    const uint32_t W = atoi(argv[2]), H = atoi(argv[3]), spp = atoi(argv[4]);
    const int bl = atoi(argv[5]), ml = atoi(argv[6]);
    const uint32_t step = argc > 7 ? atoi(argv[7]) : 1, frame = argc > 8 ? atoi(argv[8]) : 0;
    const int defer = argc > 9 ? atoi(argv[9]) : 32;
    if (64 % spp) { fprintf(stderr, "spp must divide 64\n"); return 2; }
    mm_uniform u;  /* the default camera (mm_uniform_default), written beside the scene by dump_scene.py */
    {
        char up[4096];
        snprintf(up, sizeof(up), "%s.uni", argv[1]);
        FILE* f = fopen(up, "rb");
        if (!f || fread(&u, sizeof(u), 1, f) != 1) { fprintf(stderr, "cannot read %s\n", up); return 1; }
        fclose(f);
        if ((uint32_t)u.view_w != W || (uint32_t)u.view_h != H) { fprintf(stderr, "uniform is not %ux%u\n", W, H); return 1; }
    }
    const uint32_t ppc = 64 / spp;  /* pixels per chunk */
    uint64_t chunks = 0, deferred_chunks = 0, pixels = 0, staged_pixels = 0, parked = 0, paths = 0, rays = 0;
    uint64_t hist_n[64] = {0};
#pragma omp parallel for schedule(dynamic, 1) reduction(+ : chunks, deferred_chunks, pixels, staged_pixels, parked, paths, rays)
    for (uint32_t y = 0; y < H; y += step) {
        uint64_t hloc[64] = {0};
        for (uint32_t x0 = 0; x0 < W; x0 += ppc) {
            uint32_t q[64];
            for (uint32_t l = 0; l < 64; ++l) {
                const uint32_t px = x0 + l / spp, smp = l % spp;
                if (px >= W) { q[l] = 0; continue; }
                const uint32_t pixel = y * W + px;
                uint32_t seed = oracle_tile_seed(pixel, smp, frame);
                const v3 d0 = primary_dir(&u, px, y);
                const v3 d = jittered_dir(d0, &seed);
                uint64_t r = 0;
                trav_t tr = {0, 0, 0};
                (void)trace_path(&S, ld3(u.cam.center), d, seed, bl, ml, &r, &tr);
                q[l] = (uint32_t)r;
                rays += r;
                paths++;
            }
            /* the first bounce n >= 1 at whose top 1..defer lanes are live */
            int dn = -1;
            uint32_t qmax = 0;
            for (uint32_t l = 0; l < 64; ++l) qmax = q[l] > qmax ? q[l] : qmax;
            for (uint32_t n = 1; n < qmax; ++n) {
                uint32_t live = 0;
                for (uint32_t l = 0; l < 64; ++l) live += q[l] > n;
                if (live >= 1 && live <= (uint32_t)defer) { dn = (int)n; break; }
            }
            chunks++;
            pixels += ppc;
            if (dn < 0) continue;
            deferred_chunks++;
            hloc[dn < 63 ? dn : 63]++;
            for (uint32_t p = 0; p < ppc; ++p) {
                uint32_t any = 0;
                for (uint32_t s = 0; s < spp; ++s) {
                    const uint32_t l = p * spp + s;
                    if (q[l] > (uint32_t)dn) { any = 1; parked++; }
                }
                staged_pixels += any;
            }
        }
#pragma omp critical
        for (int i = 0; i < 64; ++i) hist_n[i] += hloc[i];
    }
    const double sf = (double)staged_pixels / pixels;
    printf("{\"W\": %u, \"H\": %u, \"spp\": %u, \"bounce_limit\": %d, \"mirror_limit\": %d, \"row_step\": %u, "
           "\"frame\": %u, \"defer_lanes\": %d,\n", W, H, spp, bl, ml, step, frame, defer);
    printf(" \"paths\": %llu, \"rays\": %llu, \"chunks\": %llu, \"chunks_that_defer\": %llu, \"parked_paths\": %llu,\n",
           (unsigned long long)paths, (unsigned long long)rays, (unsigned long long)chunks,
           (unsigned long long)deferred_chunks, (unsigned long long)parked);
    printf(" \"pixels\": %llu, \"pixels_with_a_parked_sample\": %llu, \"staged_pixel_fraction\": %.4f,\n",
           (unsigned long long)pixels, (unsigned long long)staged_pixels, sf);
    printf(" \"defer_bounce_histogram\": [");
    for (int i = 0; i < 64; ++i) printf("%s%llu", i ? ", " : "", (unsigned long long)hist_n[i]);
    printf("]}\n");
    return 0;
}
