/* Writes the Keras-layout HDF5 weight fixtures of tests/test_formats.py with
 * the real HDF5 C library (the image's /opt/conda HDF5 1.10.6, the library
 * h5py wraps), so the repository's pure-Python HDF5 reader is pinned against
 * files produced by HDF5 itself.  Layout = keras 2.3.1 save_weights_to_hdf5_group
 * (engine/saving.py): root attrs layer_names / backend / keras_version
 * (fixed-length byte strings), one group per layer with attr weight_names and
 * the datasets at <layer>/<weight_name> (e.g. conv1/conv1/kernel:0).
 * Values: v[i] = sin(0.37*i + 1.3*L + 0.11*W) (layer L, weight W, flat i).
 * Build/run: tests/golden/h5src/make_h5_fixtures.sh */
#include <hdf5.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static void str_attr_array(hid_t loc, const char* name, const char** v, int n) {
    size_t len = 1;
    for (int i = 0; i < n; ++i) if (strlen(v[i]) > len) len = strlen(v[i]);
    char* buf = calloc((size_t)n, len);
    for (int i = 0; i < n; ++i) memcpy(buf + i * len, v[i], strlen(v[i]));
    hid_t t = H5Tcopy(H5T_C_S1);
    H5Tset_size(t, len);
    H5Tset_strpad(t, H5T_STR_NULLPAD);
    hsize_t d = (hsize_t)n;
    hid_t sp = H5Screate_simple(1, &d, NULL);
    hid_t a = H5Acreate2(loc, name, t, sp, H5P_DEFAULT, H5P_DEFAULT);
    H5Awrite(a, t, buf);
    H5Aclose(a); H5Sclose(sp); H5Tclose(t); free(buf);
}

static void str_attr_scalar(hid_t loc, const char* name, const char* v) {
    hid_t t = H5Tcopy(H5T_C_S1);
    H5Tset_size(t, strlen(v));
    H5Tset_strpad(t, H5T_STR_NULLPAD);
    hid_t sp = H5Screate(H5S_SCALAR);
    hid_t a = H5Acreate2(loc, name, t, sp, H5P_DEFAULT, H5P_DEFAULT);
    H5Awrite(a, t, v);
    H5Aclose(a); H5Sclose(sp); H5Tclose(t);
}

typedef struct { const char* layer; int nw; const char* wn[4]; int rank[4]; hsize_t dims[4][5]; } Layer;

static void write_weights(hid_t f, hid_t root, const Layer* L, int nl, hid_t dcpl, hid_t ftype) {
    const char* names[64];
    for (int l = 0; l < nl; ++l) names[l] = L[l].layer;
    str_attr_array(root, "layer_names", names, nl);
    str_attr_scalar(root, "backend", "tensorflow");
    str_attr_scalar(root, "keras_version", "2.3.1");
    for (int l = 0; l < nl; ++l) {
        hid_t g = H5Gcreate2(root, L[l].layer, H5P_DEFAULT, H5P_DEFAULT, H5P_DEFAULT);
        char full[4][128];
        const char* wn[4];
        for (int w = 0; w < L[l].nw; ++w) {
            snprintf(full[w], sizeof full[w], "%s/%s", L[l].layer, L[l].wn[w]);
            wn[w] = full[w];
        }
        str_attr_array(g, "weight_names", wn, L[l].nw);
        for (int w = 0; w < L[l].nw; ++w) {
            hsize_t n = 1;
            for (int r = 0; r < L[l].rank[w]; ++r) n *= L[l].dims[w][r];
            float* v = malloc(n * sizeof(float));
            for (hsize_t i = 0; i < n; ++i) v[i] = (float)sin(0.37 * (double)i + 1.3 * l + 0.11 * w);
            hid_t sp = H5Screate_simple(L[l].rank[w], L[l].dims[w], NULL);
            hid_t lcpl = H5Pcreate(H5P_LINK_CREATE);
            H5Pset_create_intermediate_group(lcpl, 1);
            hid_t d = H5Dcreate2(g, full[w], ftype, sp, lcpl, dcpl, H5P_DEFAULT);
            H5Dwrite(d, H5T_NATIVE_FLOAT, H5S_ALL, H5S_ALL, H5P_DEFAULT, v);
            H5Dclose(d); H5Pclose(lcpl); H5Sclose(sp); free(v);
        }
        H5Gclose(g);
    }
}

int main(int argc, char** argv) {
    const char* dir = argc > 1 ? argv[1] : ".";
    char path[512];
    /* the tiny RPN-like layer set the test builds on a ParamStore */
    Layer L[] = {
        {"conv1", 2, {"kernel:0", "bias:0"}, {5, 1}, {{3, 3, 3, 1, 4}, {4}}},
        {"bn_conv1", 4, {"gamma:0", "beta:0", "moving_mean:0", "moving_variance:0"}, {1, 1, 1, 1},
         {{4}, {4}, {4}, {4}}},
        {"rpn_conv_shared1", 2, {"kernel:0", "bias:0"}, {5, 1}, {{3, 3, 3, 4, 8}, {8}}},
        {"mrcnn_class_logits", 2, {"kernel:0", "bias:0"}, {2, 1}, {{8, 3}, {3}}},
        {"mrcnn_mask_deconv", 2, {"kernel:0", "bias:0"}, {5, 1}, {{2, 2, 2, 8, 4}, {8}}},
    };
    const int nl = sizeof L / sizeof L[0];
    /* 1: h5py defaults (libver earliest: superblock 0, v1 object headers,
     *    symbol-table groups), contiguous float32 little-endian */
    snprintf(path, sizeof path, "%s/keras_weights_v0.h5", dir);
    hid_t f = H5Fcreate(path, H5F_ACC_TRUNC, H5P_DEFAULT, H5P_DEFAULT);
    write_weights(f, f, L, nl, H5P_DEFAULT, H5T_IEEE_F32LE);
    H5Fclose(f);
    /* 2: full-model save layout (model_weights group), latest format
     *    (superblock 3, v2 object headers, link messages), chunked + deflate
     *    + shuffle, big-endian storage */
    snprintf(path, sizeof path, "%s/keras_model_latest.h5", dir);
    hid_t fapl = H5Pcreate(H5P_FILE_ACCESS);
    H5Pset_libver_bounds(fapl, H5F_LIBVER_LATEST, H5F_LIBVER_LATEST);
    f = H5Fcreate(path, H5F_ACC_TRUNC, H5P_DEFAULT, fapl);
    hid_t mw = H5Gcreate2(f, "model_weights", H5P_DEFAULT, H5P_DEFAULT, H5P_DEFAULT);
    hid_t dcpl = H5Pcreate(H5P_DATASET_CREATE);
    hsize_t ch[5] = {2, 2, 2, 2, 2};
    (void)ch;
    write_weights(f, mw, L, nl, H5P_DEFAULT, H5T_IEEE_F32BE);
    /* a chunked, shuffled, deflated dataset next to the weights */
    hsize_t dd[3] = {5, 6, 7}, cd[3] = {2, 3, 4};
    H5Pset_chunk(dcpl, 3, cd);
    H5Pset_shuffle(dcpl);
    H5Pset_deflate(dcpl, 4);
    float v[210];
    for (int i = 0; i < 210; ++i) v[i] = (float)(i * 0.5 - 7.0);
    hid_t sp = H5Screate_simple(3, dd, NULL);
    hid_t d = H5Dcreate2(f, "chunked_deflate", H5T_IEEE_F32LE, sp, H5P_DEFAULT, dcpl, H5P_DEFAULT);
    H5Dwrite(d, H5T_NATIVE_FLOAT, H5S_ALL, H5S_ALL, H5P_DEFAULT, v);
    H5Dclose(d); H5Sclose(sp);
    H5Gclose(mw); H5Pclose(dcpl); H5Pclose(fapl);
    H5Fclose(f);
    /* 3: a wide model (300 layers -> multi-level symbol-table B-tree, layer
     *    names attribute split into layer_names0/1 as keras does above 64 KiB
     *    is emulated by a second attribute), int32 + float64 datasets,
     *    chunked-without-filters, earliest format */
    snprintf(path, sizeof path, "%s/wide_v0.h5", dir);
    f = H5Fcreate(path, H5F_ACC_TRUNC, H5P_DEFAULT, H5P_DEFAULT);
    const char* part0[150]; const char* part1[150];
    char nm[300][32];
    for (int i = 0; i < 300; ++i) snprintf(nm[i], 32, "layer_%03d", i);
    for (int i = 0; i < 150; ++i) { part0[i] = nm[i]; part1[i] = nm[150 + i]; }
    str_attr_array(f, "layer_names0", part0, 150);
    str_attr_array(f, "layer_names1", part1, 150);
    for (int i = 0; i < 300; ++i) {
        hid_t g = H5Gcreate2(f, nm[i], H5P_DEFAULT, H5P_DEFAULT, H5P_DEFAULT);
        int32_t iv[3] = {i, -i, 7 * i};
        hsize_t n3 = 3;
        sp = H5Screate_simple(1, &n3, NULL);
        d = H5Dcreate2(g, "ints", H5T_STD_I32LE, sp, H5P_DEFAULT, H5P_DEFAULT, H5P_DEFAULT);
        H5Dwrite(d, H5T_NATIVE_INT32, H5S_ALL, H5S_ALL, H5P_DEFAULT, iv);
        H5Dclose(d); H5Sclose(sp);
        H5Gclose(g);
    }
    hsize_t d2[2] = {9, 10}, c2[2] = {4, 4};
    double dv[90];
    for (int i = 0; i < 90; ++i) dv[i] = 1.0 / (i + 1);
    dcpl = H5Pcreate(H5P_DATASET_CREATE);
    H5Pset_chunk(dcpl, 2, c2);
    sp = H5Screate_simple(2, d2, NULL);
    d = H5Dcreate2(f, "chunked_f64", H5T_IEEE_F64LE, sp, H5P_DEFAULT, dcpl, H5P_DEFAULT);
    H5Dwrite(d, H5T_NATIVE_DOUBLE, H5S_ALL, H5S_ALL, H5P_DEFAULT, dv);
    H5Dclose(d); H5Sclose(sp); H5Pclose(dcpl);
    H5Fclose(f);
    return 0;
}
