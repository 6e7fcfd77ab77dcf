// image_io.hpp -- grayscale image I/O for the interactive driver.
// PGM (P5, 8-bit) is always available.  JPEG goes through libjpeg when the
// driver is built with -DHPDCT_WITH_JPEG (the reference's load_jpeg_as_matrix /
// save_grayscale_jpeg, utils.cu:38-147, are libjpeg-based too); a colour JPEG
// is converted to grayscale on decode (the reference instead overflows its
// float buffer, main_newAppr.cu:46-47).
#pragma once

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#ifdef HPDCT_WITH_JPEG
#include <jpeglib.h>
#endif

namespace hpdct_io {

inline bool ends_with(const std::string& s, const char* suf) {
    const size_t n = strlen(suf);
    if (s.size() < n) return false;
    for (size_t i = 0; i < n; ++i)
        if (tolower((unsigned char)s[s.size() - n + i]) != suf[i]) return false;
    return true;
}

inline bool is_jpeg(const std::string& p) { return ends_with(p, ".jpg") || ends_with(p, ".jpeg"); }

// Largest accepted header field: 2^24 px per side, and w * h below 2^31.
constexpr int kPgmMaxToken = 1 << 24;

inline int pgm_token(FILE* f) {
    int c = fgetc(f);
    while (c == '#' || c == ' ' || c == '\n' || c == '\r' || c == '\t') {
        if (c == '#')
            while (c != '\n' && c != EOF) c = fgetc(f);
        c = fgetc(f);
    }
    int v = 0;
    bool any = false;
    while (c >= '0' && c <= '9') {
        if (v > kPgmMaxToken / 10) return -1;  // no int overflow on a hostile header (UBSan-checked)
        v = v * 10 + (c - '0');
        any = true;
        c = fgetc(f);
    }
    return any ? v : -1;
}

inline bool load_pgm(const std::string& path, std::vector<uint8_t>& px, int& w, int& h) {
    FILE* f = fopen(path.c_str(), "rb");
    if (!f) return false;
    char magic[3] = {0, 0, 0};
    if (fread(magic, 1, 2, f) != 2 || magic[0] != 'P' || magic[1] != '5') {
        fclose(f);
        return false;
    }
    w = pgm_token(f);
    h = pgm_token(f);
    const int maxv = pgm_token(f);
    if (w <= 0 || h <= 0 || maxv <= 0 || maxv > 255 || (int64_t)w * h >= ((int64_t)1 << 31)) {
        fclose(f);
        return false;
    }
    px.resize((size_t)w * h);
    const bool ok = fread(px.data(), 1, px.size(), f) == px.size();
    fclose(f);
    return ok;
}

inline bool save_pgm(const std::string& path, const uint8_t* px, int w, int h) {
    FILE* f = fopen(path.c_str(), "wb");
    if (!f) return false;
    fprintf(f, "P5\n%d %d\n255\n", w, h);
    const bool ok = fwrite(px, 1, (size_t)w * h, f) == (size_t)w * h;
    fclose(f);
    return ok;
}

#ifdef HPDCT_WITH_JPEG
inline bool load_jpeg(const std::string& path, std::vector<uint8_t>& px, int& w, int& h) {
    FILE* f = fopen(path.c_str(), "rb");
    if (!f) return false;
    jpeg_decompress_struct cinfo;
    jpeg_error_mgr jerr;
    cinfo.err = jpeg_std_error(&jerr);
    jpeg_create_decompress(&cinfo);
    jpeg_stdio_src(&cinfo, f);
    jpeg_read_header(&cinfo, TRUE);
    cinfo.out_color_space = JCS_GRAYSCALE;
    jpeg_start_decompress(&cinfo);
    w = (int)cinfo.output_width;
    h = (int)cinfo.output_height;
    px.resize((size_t)w * h);
    while (cinfo.output_scanline < cinfo.output_height) {
        JSAMPROW row = px.data() + (size_t)cinfo.output_scanline * w;
        jpeg_read_scanlines(&cinfo, &row, 1);
    }
    jpeg_finish_decompress(&cinfo);
    jpeg_destroy_decompress(&cinfo);
    fclose(f);
    return true;
}

inline bool save_jpeg(const std::string& path, const uint8_t* px, int w, int h, int quality) {
    FILE* f = fopen(path.c_str(), "wb");
    if (!f) return false;
    jpeg_compress_struct cinfo;
    jpeg_error_mgr jerr;
    cinfo.err = jpeg_std_error(&jerr);
    jpeg_create_compress(&cinfo);
    jpeg_stdio_dest(&cinfo, f);
    cinfo.image_width = w;
    cinfo.image_height = h;
    cinfo.input_components = 1;
    cinfo.in_color_space = JCS_GRAYSCALE;
    jpeg_set_defaults(&cinfo);
    jpeg_set_quality(&cinfo, quality, TRUE);
    jpeg_start_compress(&cinfo, TRUE);
    while (cinfo.next_scanline < cinfo.image_height) {
        JSAMPROW row = const_cast<uint8_t*>(px) + (size_t)cinfo.next_scanline * w;
        jpeg_write_scanlines(&cinfo, &row, 1);
    }
    jpeg_finish_compress(&cinfo);
    jpeg_destroy_compress(&cinfo);
    fclose(f);
    return true;
}
#endif

inline bool load_gray(const std::string& path, std::vector<uint8_t>& px, int& w, int& h) {
    if (is_jpeg(path)) {
#ifdef HPDCT_WITH_JPEG
        return load_jpeg(path, px, w, h);
#else
        fprintf(stderr, "Error: built without libjpeg; use a .pgm image\n");
        return false;
#endif
    }
    return load_pgm(path, px, w, h);
}

inline bool save_gray(const std::string& path, const uint8_t* px, int w, int h, int quality) {
    if (is_jpeg(path)) {
#ifdef HPDCT_WITH_JPEG
        return save_jpeg(path, px, w, h, quality);
#else
        fprintf(stderr, "Error: built without libjpeg; use a .pgm image\n");
        return false;
#endif
    }
    (void)quality;
    return save_pgm(path, px, w, h);
}

}  // namespace hpdct_io
