// png_codec.cpp -- PNG decode/encode on zlib for matcaps and rendered frames.
//
// Replaces the vendored lodepng (reference src/common/lodepng.cpp) as used by
// Image::loadPNG (src/neuralUtils/image.cu:36-65: decode to 8-bit RGBA, pack
// a<<24|b<<16|g<<8|r) and Image::savePNG (:67-110: with doFlip the byte stream is
// reversed, i.e. the frame is rotated 180 degrees -- quirk Q9).  Decoding follows
// lodepng's RGBA8 conversion: RGB -> alpha 255, grey -> r=g=b, palette via PLTE
// (+tRNS), 16-bit channels keep their high byte, tRNS colour keys -> alpha 0.
// Interlaced (Adam7) images are rejected.
#include "nr_internal.h"

#include <zlib.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

namespace nr {
namespace {

uint32_t be32(const uint8_t *p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }
void put32(std::vector<uint8_t> &v, uint32_t x) {
    v.push_back(x >> 24); v.push_back(x >> 16); v.push_back(x >> 8); v.push_back(x);
}

int paeth(int a, int b, int c) {
    int p = a + b - c, pa = abs(p - a), pb = abs(p - b), pc = abs(p - c);
    if (pa <= pb && pa <= pc) return a;
    if (pb <= pc) return b;
    return c;
}

}  // namespace

int png_decode(const char *path, std::vector<uint32_t> &rgba, int &w, int &h, std::string &err) {
    FILE *fp = fopen(path, "rb");
    if (!fp) { err = std::string("cannot open ") + path; return NR_E_IO; }
    std::vector<uint8_t> f;
    uint8_t buf[1 << 16];
    size_t n;
    while ((n = fread(buf, 1, sizeof buf, fp)) > 0) f.insert(f.end(), buf, buf + n);
    fclose(fp);
    static const uint8_t sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
    if (f.size() < 8 || memcmp(f.data(), sig, 8) != 0) { err = "not a PNG file"; return NR_E_FORMAT; }
    size_t p = 8;
    uint32_t W = 0, H = 0;
    int depth = 0, ctype = -1, interlace = 0;
    std::vector<uint8_t> idat, plte, trns;
    bool seen_iend = false;
    while (p + 12 <= f.size() && !seen_iend) {
        uint32_t len = be32(&f[p]);
        if (len > f.size() - p - 12) { err = "truncated PNG chunk"; return NR_E_FORMAT; }
        const uint8_t *type = &f[p + 4], *data = &f[p + 8];
        if (!memcmp(type, "IHDR", 4)) {
            if (len < 13) { err = "bad IHDR"; return NR_E_FORMAT; }
            W = be32(data); H = be32(data + 4);
            depth = data[8]; ctype = data[9]; interlace = data[12];
            if (data[10] != 0 || data[11] != 0) { err = "unknown PNG compression/filter method"; return NR_E_FORMAT; }
        } else if (!memcmp(type, "IDAT", 4)) {
            idat.insert(idat.end(), data, data + len);
        } else if (!memcmp(type, "PLTE", 4)) {
            plte.assign(data, data + len);
        } else if (!memcmp(type, "tRNS", 4)) {
            trns.assign(data, data + len);
        } else if (!memcmp(type, "IEND", 4)) {
            seen_iend = true;
        }
        p += 12 + len;
    }
    if (W == 0 || H == 0 || W > (1u << 15) || H > (1u << 15)) { err = "bad PNG size"; return NR_E_FORMAT; }
    if (interlace) { err = "interlaced PNG unsupported"; return NR_E_FORMAT; }
    int chans;
    switch (ctype) {
        case 0: chans = 1; break;
        case 2: chans = 3; break;
        case 3: chans = 1; break;
        case 4: chans = 2; break;
        case 6: chans = 4; break;
        default: err = "bad PNG colour type"; return NR_E_FORMAT;
    }
    bool ok_depth = (depth == 8 || depth == 16) || (ctype == 3 && (depth == 1 || depth == 2 || depth == 4)) ||
                    (ctype == 0 && (depth == 1 || depth == 2 || depth == 4));
    if (!ok_depth) { err = "unsupported PNG bit depth"; return NR_E_FORMAT; }
    if (ctype == 3 && plte.empty()) { err = "palette PNG without PLTE"; return NR_E_FORMAT; }
    size_t bits_pp = (size_t)chans * depth;
    size_t stride = (W * bits_pp + 7) / 8;
    size_t bpp = (bits_pp + 7) / 8;
    std::vector<uint8_t> raw((stride + 1) * H);
    uLongf rawlen = raw.size();
    z_stream zs;
    memset(&zs, 0, sizeof zs);
    if (inflateInit(&zs) != Z_OK) { err = "zlib init failed"; return NR_E_FORMAT; }
    zs.next_in = idat.data(); zs.avail_in = (uInt)idat.size();
    zs.next_out = raw.data(); zs.avail_out = (uInt)rawlen;
    int zr = inflate(&zs, Z_FINISH);
    size_t produced = rawlen - zs.avail_out;
    inflateEnd(&zs);
    if ((zr != Z_STREAM_END && zr != Z_BUF_ERROR) || produced != raw.size()) {
        err = "corrupt PNG image data"; return NR_E_FORMAT;
    }
    // unfilter in place
    std::vector<uint8_t> img(stride * H);
    for (uint32_t y = 0; y < H; ++y) {
        uint8_t ft = raw[y * (stride + 1)];
        const uint8_t *src = &raw[y * (stride + 1) + 1];
        uint8_t *dst = &img[y * stride];
        const uint8_t *up = y ? &img[(y - 1) * stride] : nullptr;
        for (size_t i = 0; i < stride; ++i) {
            int a = i >= bpp ? dst[i - bpp] : 0;
            int b = up ? up[i] : 0;
            int c = (up && i >= bpp) ? up[i - bpp] : 0;
            int v = src[i];
            switch (ft) {
                case 0: break;
                case 1: v += a; break;
                case 2: v += b; break;
                case 3: v += (a + b) >> 1; break;
                case 4: v += paeth(a, b, c); break;
                default: err = "bad PNG filter type"; return NR_E_FORMAT;
            }
            dst[i] = (uint8_t)v;
        }
    }
    w = (int)W; h = (int)H;
    rgba.assign((size_t)W * H, 0);
    auto sample = [&](const uint8_t *row, uint32_t x, int c) -> unsigned {
        // returns the 8-bit value (high byte for 16-bit) and, for sub-byte depths, the raw index/grey
        if (depth == 8) return row[x * chans + c];
        if (depth == 16) return row[(x * chans + c) * 2];
        size_t bit = (size_t)x * depth;
        unsigned v = (row[bit / 8] >> (8 - depth - (bit % 8))) & ((1u << depth) - 1);
        return v;
    };
    auto raw16 = [&](const uint8_t *row, uint32_t x, int c) -> unsigned {
        if (depth == 16) return (unsigned)row[(x * chans + c) * 2] << 8 | row[(x * chans + c) * 2 + 1];
        return sample(row, x, c);
    };
    for (uint32_t y = 0; y < H; ++y) {
        const uint8_t *row = &img[y * stride];
        for (uint32_t x = 0; x < W; ++x) {
            unsigned r, g, b, a = 255;
            if (ctype == 3) {
                unsigned idx = sample(row, x, 0);
                if (idx * 3 + 2 >= plte.size()) { r = g = b = 0; a = 0; }  // lodepng: out-of-palette -> error; use black
                else { r = plte[idx * 3]; g = plte[idx * 3 + 1]; b = plte[idx * 3 + 2]; }
                if (idx < trns.size()) a = trns[idx];
            } else if (ctype == 0 || ctype == 4) {
                unsigned v = sample(row, x, 0);
                if (depth < 8) v = v * 255 / ((1u << depth) - 1);
                r = g = b = v;
                if (ctype == 4) a = sample(row, x, 1);
                else if (trns.size() >= 2) {
                    unsigned key = (unsigned)trns[0] << 8 | trns[1];
                    if (raw16(row, x, 0) == key) a = 0;
                }
            } else {
                r = sample(row, x, 0); g = sample(row, x, 1); b = sample(row, x, 2);
                if (ctype == 6) a = sample(row, x, 3);
                else if (trns.size() >= 6) {
                    unsigned kr = (unsigned)trns[0] << 8 | trns[1], kg = (unsigned)trns[2] << 8 | trns[3],
                             kb = (unsigned)trns[4] << 8 | trns[5];
                    if (raw16(row, x, 0) == kr && raw16(row, x, 1) == kg && raw16(row, x, 2) == kb) a = 0;
                }
            }
            rgba[(size_t)y * W + x] = (a << 24) | (b << 16) | (g << 8) | r;   // image.cu:57-58
        }
    }
    return NR_OK;
}

int png_encode(const char *path, const uint32_t *rgba, int w, int h, int flip, std::string &err) {
    if (w <= 0 || h <= 0) { err = "bad image size"; return NR_E_INVALID; }
    size_t npx = (size_t)w * h;
    // image.cu:75-98: per pixel push a,b,g,r then reverse the whole stream when flipping,
    // which yields r,g,b,a bytes with pixel order reversed (180 deg rotation).
    std::vector<uint8_t> bytes(npx * 4);
    for (size_t i = 0; i < npx; ++i) {
        uint32_t c = flip ? rgba[npx - 1 - i] : rgba[i];
        bytes[4 * i] = c & 0xff; bytes[4 * i + 1] = (c >> 8) & 0xff;
        bytes[4 * i + 2] = (c >> 16) & 0xff; bytes[4 * i + 3] = (c >> 24) & 0xff;
    }
    std::vector<uint8_t> raw((size_t)(w * 4 + 1) * h);
    for (int y = 0; y < h; ++y) {
        raw[(size_t)y * (w * 4 + 1)] = 0;
        memcpy(&raw[(size_t)y * (w * 4 + 1) + 1], &bytes[(size_t)y * w * 4], (size_t)w * 4);
    }
    uLongf clen = compressBound(raw.size());
    std::vector<uint8_t> comp(clen);
    if (compress2(comp.data(), &clen, raw.data(), raw.size(), 6) != Z_OK) { err = "zlib compress failed"; return NR_E_FORMAT; }
    comp.resize(clen);
    std::vector<uint8_t> out = {137, 80, 78, 71, 13, 10, 26, 10};
    auto chunk = [&](const char *type, const uint8_t *d, size_t len) {
        put32(out, (uint32_t)len);
        size_t start = out.size();
        out.insert(out.end(), type, type + 4);
        out.insert(out.end(), d, d + len);
        uint32_t crc = (uint32_t)crc32(0, &out[start], (uInt)(len + 4));
        put32(out, crc);
    };
    std::vector<uint8_t> ihdr;
    put32(ihdr, (uint32_t)w); put32(ihdr, (uint32_t)h);
    ihdr.push_back(8); ihdr.push_back(6); ihdr.push_back(0); ihdr.push_back(0); ihdr.push_back(0);
    chunk("IHDR", ihdr.data(), ihdr.size());
    chunk("IDAT", comp.data(), comp.size());
    chunk("IEND", nullptr, 0);
    FILE *fp = fopen(path, "wb");
    if (!fp) { err = std::string("cannot write ") + path; return NR_E_IO; }
    size_t wr = fwrite(out.data(), 1, out.size(), fp);
    fclose(fp);
    if (wr != out.size()) { err = "short write"; return NR_E_IO; }
    return NR_OK;
}

int ppm_encode(const char *path, const uint32_t *rgba, int w, int h, std::string &err) {
    FILE *fp = fopen(path, "wb");
    if (!fp) { err = std::string("cannot write ") + path; return NR_E_IO; }
    // helper_image.h:310-328 (sdkSavePPM4ub): "P6\n<w>\n<h>\n255\n", RGB, row 0 first
    fprintf(fp, "P6\n%d\n%d\n255\n", w, h);
    std::vector<uint8_t> row((size_t)w * 3);
    for (int y = 0; y < h; ++y) {
        for (int x = 0; x < w; ++x) {
            uint32_t c = rgba[(size_t)y * w + x];
            row[3 * x] = c & 0xff; row[3 * x + 1] = (c >> 8) & 0xff; row[3 * x + 2] = (c >> 16) & 0xff;
        }
        fwrite(row.data(), 1, row.size(), fp);
    }
    fclose(fp);
    return NR_OK;
}

}  // namespace nr
