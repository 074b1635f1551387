// image_io.cpp — PPM / PNG writers and host RGBA8 quantisation (include/mm_io.h).
#include "mm_io.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

namespace {

uint32_t crc_table[256];
bool crc_ready = false;

void crc_init() {
    for (uint32_t n = 0; n < 256; ++n) {
        uint32_t c = n;
        for (int k = 0; k < 8; ++k) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
        crc_table[n] = c;
    }
    crc_ready = true;
}

uint32_t crc32(uint32_t crc, const uint8_t* p, size_t n) {
    crc = ~crc;
    for (size_t i = 0; i < n; ++i) crc = crc_table[(crc ^ p[i]) & 0xFFu] ^ (crc >> 8);
    return ~crc;
}

void put_be32(std::vector<uint8_t>& v, uint32_t x) {
    v.push_back((uint8_t)(x >> 24)); v.push_back((uint8_t)(x >> 16));
    v.push_back((uint8_t)(x >> 8)); v.push_back((uint8_t)x);
}

void chunk(std::vector<uint8_t>& out, const char type[4], const std::vector<uint8_t>& data) {
    put_be32(out, (uint32_t)data.size());
    const size_t start = out.size();
    out.insert(out.end(), type, type + 4);
    out.insert(out.end(), data.begin(), data.end());
    put_be32(out, crc32(0, out.data() + start, out.size() - start));
}

int write_all(const char* path, const uint8_t* p, size_t n) {
    FILE* f = std::fopen(path, "wb");
    if (!f) return MM_ERR_INVALID;
    const size_t w = std::fwrite(p, 1, n, f);
    const int rc = std::fclose(f);
    return (w == n && rc == 0) ? MM_OK : MM_ERR_INVALID;
}

}  // namespace

extern "C" {

int mm_write_ppm(const char* path, const uint8_t* rgba8, uint32_t w, uint32_t h) {
    if (!path || !rgba8 || w == 0 || h == 0) return MM_ERR_INVALID;
    char hdr[64];
    const int hn = std::snprintf(hdr, sizeof(hdr), "P6\n%u %u\n255\n", w, h);
    std::vector<uint8_t> out(hdr, hdr + hn);
    out.reserve(out.size() + (size_t)w * h * 3);
    for (size_t i = 0; i < (size_t)w * h; ++i) out.insert(out.end(), rgba8 + 4 * i, rgba8 + 4 * i + 3);
    return write_all(path, out.data(), out.size());
}

int mm_write_png(const char* path, const uint8_t* rgba8, uint32_t w, uint32_t h) {
    if (!path || !rgba8 || w == 0 || h == 0 || w > 0x7FFFFFFFu || h > 0x7FFFFFFFu) return MM_ERR_INVALID;
    if (!crc_ready) crc_init();
    // raw scanlines: filter byte 0 + 4w bytes
    const size_t row = 1 + 4 * (size_t)w;
    std::vector<uint8_t> raw(row * h);
    for (uint32_t y = 0; y < h; ++y) {
        raw[row * y] = 0;
        std::memcpy(&raw[row * y + 1], rgba8 + 4 * (size_t)w * y, 4 * (size_t)w);
    }
    // zlib stream: CMF/FLG (deflate, 32K window, no dict, check bits), stored blocks, Adler-32
    std::vector<uint8_t> z{0x78, 0x01};
    size_t pos = 0;
    do {
        const size_t n = std::min<size_t>(65535, raw.size() - pos);
        const bool last = pos + n == raw.size();
        z.push_back(last ? 1 : 0);
        z.push_back((uint8_t)n); z.push_back((uint8_t)(n >> 8));
        z.push_back((uint8_t)~n); z.push_back((uint8_t)(~n >> 8));
        z.insert(z.end(), raw.begin() + pos, raw.begin() + pos + n);
        pos += n;
    } while (pos < raw.size());
    uint32_t a = 1, b = 0;
    for (uint8_t v : raw) { a = (a + v) % 65521u; b = (b + a) % 65521u; }
    put_be32(z, (b << 16) | a);
    std::vector<uint8_t> out{0x89, 'P', 'N', 'G', '\r', '\n', 0x1A, '\n'};
    std::vector<uint8_t> ihdr;
    put_be32(ihdr, w);
    put_be32(ihdr, h);
    ihdr.insert(ihdr.end(), {8, 6, 0, 0, 0});  // depth 8, RGBA, deflate, filter 0, no interlace
    chunk(out, "IHDR", ihdr);
    chunk(out, "IDAT", z);
    chunk(out, "IEND", {});
    return write_all(path, out.data(), out.size());
}

void mm_quantize_rgba8_host(const float* rgba, uint8_t* rgba8, uint64_t n_pixels) {
    if (!rgba || !rgba8) return;
    for (uint64_t i = 0; i < 4 * n_pixels; ++i) {
        const float x = std::fmin(std::fmax(rgba[i], 0.0f), 1.0f);  // NaN -> 0, as fmaxf on the device
        rgba8[i] = (uint8_t)std::nearbyint(x * 255.0f);
    }
}

}  // extern "C"
