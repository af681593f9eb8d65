/* Writes the multi-page TIFF fixtures of tests/test_formats.py with libtiff
 * (the image's /opt/conda libtiff), pinning m3d.tiff against files written by
 * the reference TIFF library.  Values: v(z,y,x) = (7z + 3y + x) mod 251 for
 * 8-bit, (1000z + 17y + 5x) for 16-bit.
 * Build/run: tests/golden/h5src/make_tiff_fixtures.sh */
#include <stdint.h>
#include <stdio.h>
#include <tiffio.h>

static int write_stack(const char* path, const char* mode, int bps, int Z, int Y, int X, int comp,
                       int pred, int rps) {
    TIFF* t = TIFFOpen(path, mode);
    if (!t) return 1;
    uint8_t row[4096];
    for (int z = 0; z < Z; ++z) {
        TIFFSetField(t, TIFFTAG_IMAGEWIDTH, X);
        TIFFSetField(t, TIFFTAG_IMAGELENGTH, Y);
        TIFFSetField(t, TIFFTAG_BITSPERSAMPLE, bps);
        TIFFSetField(t, TIFFTAG_SAMPLESPERPIXEL, 1);
        TIFFSetField(t, TIFFTAG_PHOTOMETRIC, PHOTOMETRIC_MINISBLACK);
        TIFFSetField(t, TIFFTAG_PLANARCONFIG, PLANARCONFIG_CONTIG);
        TIFFSetField(t, TIFFTAG_COMPRESSION, comp);
        if (pred) TIFFSetField(t, TIFFTAG_PREDICTOR, pred);
        TIFFSetField(t, TIFFTAG_ROWSPERSTRIP, rps);
        TIFFSetField(t, TIFFTAG_SUBFILETYPE, FILETYPE_PAGE);
        TIFFSetField(t, TIFFTAG_PAGENUMBER, z, Z);
        for (int y = 0; y < Y; ++y) {
            for (int x = 0; x < X; ++x) {
                if (bps == 8) row[x] = (uint8_t)((7 * z + 3 * y + x) % 251);
                else ((uint16_t*)row)[x] = (uint16_t)(1000 * z + 17 * y + 5 * x);
            }
            if (TIFFWriteScanline(t, row, y, 0) < 0) return 2;
        }
        TIFFWriteDirectory(t);
    }
    TIFFClose(t);
    return 0;
}

int main(int argc, char** argv) {
    const char* dir = argc > 1 ? argv[1] : ".";
    char p[512];
    int rc = 0;
    snprintf(p, sizeof p, "%s/stack_u8.tif", dir);
    rc |= write_stack(p, "w", 8, 5, 7, 9, COMPRESSION_NONE, 0, 3);        /* II, uncompressed */
    snprintf(p, sizeof p, "%s/stack_u16_be_deflate.tif", dir);
    rc |= write_stack(p, "wb", 16, 4, 6, 11, COMPRESSION_ADOBE_DEFLATE, 2, 4); /* MM, deflate + predictor */
    snprintf(p, sizeof p, "%s/stack_u8_packbits_big.tif", dir);
    rc |= write_stack(p, "w8", 8, 3, 5, 6, COMPRESSION_PACKBITS, 0, 2);    /* BigTIFF, PackBits */
    return rc;
}
