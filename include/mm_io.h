/*
 * mm_io.h — on-disk formats for rendered frames (host side, no GPU needed).
 *
 * The reference only presents frames in a window (src/main.rs:888-893); an
 * offline renderer needs files.  These write the RGBA8 texture layout that
 * mm_read_framebuffer / mm_quantize_rgba8 produce (row-major, y down, 4 B per
 * texel, R first).  Self-contained: no zlib, the PNG uses stored (level-0)
 * deflate blocks, so it is byte-for-byte deterministic.
 */
#ifndef MM_IO_H
#define MM_IO_H

#include "mm_types.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Binary PPM (P6, maxval 255); alpha is dropped. */
int mm_write_ppm(const char* path, const uint8_t* rgba8, uint32_t w, uint32_t h);

/* PNG, colour type 6 (RGBA), bit depth 8, filter 0 on every row, one zlib
 * stream of stored blocks; CRC-32 and Adler-32 as the PNG / zlib specs define. */
int mm_write_png(const char* path, const uint8_t* rgba8, uint32_t w, uint32_t h);

/* Host-side twin of mm_quantize_rgba8 (the texture-write conversion:
 * round-to-nearest-even of clamp(x,0,1)*255, NaN -> 0). */
void mm_quantize_rgba8_host(const float* rgba, uint8_t* rgba8, uint64_t n_pixels);

#ifdef __cplusplus
}
#endif
#endif
