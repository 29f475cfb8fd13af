/*
 * knn_matio.c -- MAT-file (level 5 / v7) reader for knn_load_mat().
 *
 * Replaces the proprietary MATLAB MAT-API the reference links against:
 * matOpen / matGetVariable / mxGetM / mxGetN / mxGetPr / mxDestroyArray /
 * matClose (serial:40-52, 100-109; blk:64-68, 72-79, 113-116; nb:74-78,
 * 82-89, 123-126).  Supports the level-5 container written by MATLAB -v6/-v7
 * and scipy.io.savemat: uncompressed miMATRIX elements and zlib-compressed
 * miCOMPRESSED ones, either byte order, any real numeric class (converted
 * to double, as mxGetPr of a double array).  v7.3 (HDF5) files are
 * recognised and refused with KNN_ERR_UNSUPPORTED.
 */
#include "knn.h"

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>

enum {
    miINT8 = 1, miUINT8 = 2, miINT16 = 3, miUINT16 = 4, miINT32 = 5, miUINT32 = 6,
    miSINGLE = 7, miDOUBLE = 9, miINT64 = 12, miUINT64 = 13, miMATRIX = 14,
    miCOMPRESSED = 15, miUTF8 = 16, miUTF16 = 17, miUTF32 = 18
};
enum { mxCELL = 1, mxSTRUCT = 2, mxOBJECT = 3, mxCHAR = 4, mxSPARSE = 5, mxDOUBLE = 6,
       mxSINGLE = 7, mxINT8 = 8, mxUINT8 = 9, mxINT16 = 10, mxUINT16 = 11, mxINT32 = 12,
       mxUINT32 = 13, mxINT64 = 14, mxUINT64 = 15 };

typedef struct {
    const uint8_t *p;
    size_t n;
    int swap;
} buf_t;

static uint32_t rd32(const uint8_t *p, int swap)
{
    uint32_t v;
    memcpy(&v, p, 4);
    return swap ? __builtin_bswap32(v) : v;
}

/* Read one data-element tag at *off; returns payload pointer/size and the
 * offset of the next element (8-byte aligned, except after a compressed
 * element, which MATLAB does not pad). */
static int read_tag(const buf_t *b, size_t off, uint32_t *type, uint32_t *nbytes,
                    const uint8_t **data, size_t *next)
{
    if (off + 8 > b->n) return KNN_ERR_FORMAT;
    uint32_t w0 = rd32(b->p + off, b->swap);
    if (w0 >> 16) { /* small data element: 2-byte size, 2-byte type, 4 data bytes */
        *type = w0 & 0xffff;
        *nbytes = w0 >> 16;
        if (*nbytes > 4) return KNN_ERR_FORMAT;
        *data = b->p + off + 4;
        *next = off + 8;
        return KNN_OK;
    }
    *type = w0;
    *nbytes = rd32(b->p + off + 4, b->swap);
    if (off + 8 + (size_t)*nbytes > b->n) return KNN_ERR_FORMAT;
    *data = b->p + off + 8;
    size_t adv = (size_t)*nbytes;
    if (*type != miCOMPRESSED) adv = (adv + 7) & ~(size_t)7;
    *next = off + 8 + adv;
    if (*next > b->n) *next = b->n;
    return KNN_OK;
}

typedef struct {
    uint32_t cls;
    int32_t dims[2];
    int ndims;
    char name[64];
    uint32_t re_type, re_bytes;
    const uint8_t *re;
} mx_t;

/* Parse the sub-elements of a miMATRIX payload (flags, dims, name, real). */
static int parse_matrix(const uint8_t *p, size_t n, int swap, mx_t *mx, int header_only)
{
    buf_t b = {p, n, swap};
    uint32_t t, nb;
    const uint8_t *d;
    size_t off = 0, next;
    memset(mx, 0, sizeof(*mx));
    if (read_tag(&b, off, &t, &nb, &d, &next) || t != miUINT32 || nb < 8) return KNN_ERR_FORMAT;
    mx->cls = rd32(d, swap) & 0xff;
    off = next;
    if (read_tag(&b, off, &t, &nb, &d, &next) || t != miINT32 || nb < 4) return KNN_ERR_FORMAT;
    mx->ndims = (int)(nb / 4);
    /* dims are non-negative and their product must not wrap: trailing dims
     * fold into dims[1] in 64-bit, capped at INT32_MAX each */
    {
        const int32_t d0 = (int32_t)rd32(d, swap);
        int64_t d1 = mx->ndims > 1 ? (int32_t)rd32(d + 4, swap) : 1;
        if (d0 < 0 || d1 < 0) return KNN_ERR_FORMAT;
        for (int i = 2; i < mx->ndims; i++) {
            const int32_t di = (int32_t)rd32(d + 4 * i, swap);
            if (di < 0) return KNN_ERR_FORMAT;
            d1 *= di;
            if (d1 > INT32_MAX) return KNN_ERR_FORMAT;
        }
        mx->dims[0] = d0;
        mx->dims[1] = (int32_t)d1;
    }
    off = next;
    if (read_tag(&b, off, &t, &nb, &d, &next) || (t != miINT8 && t != miUTF8)) return KNN_ERR_FORMAT;
    size_t ln = nb < sizeof(mx->name) - 1 ? nb : sizeof(mx->name) - 1;
    memcpy(mx->name, d, ln);
    mx->name[ln] = 0;
    off = next;
    if (header_only) return KNN_OK;
    if (mx->cls < mxDOUBLE || mx->cls > mxUINT64) return KNN_ERR_UNSUPPORTED;
    if (read_tag(&b, off, &t, &nb, &d, &next)) return KNN_ERR_FORMAT;
    mx->re_type = t;
    mx->re_bytes = nb;
    mx->re = d;
    return KNN_OK;
}

static int elem_size(uint32_t t)
{
    switch (t) {
    case miINT8: case miUINT8: return 1;
    case miINT16: case miUINT16: return 2;
    case miINT32: case miUINT32: case miSINGLE: return 4;
    case miDOUBLE: case miINT64: case miUINT64: return 8;
    default: return 0;
    }
}

static double conv1(const uint8_t *p, uint32_t t, int swap)
{
    uint8_t tmp[8];
    int sz = elem_size(t);
    for (int i = 0; i < sz; i++) tmp[i] = swap ? p[sz - 1 - i] : p[i];
    switch (t) {
    case miINT8: return (double)(int8_t)tmp[0];
    case miUINT8: return (double)tmp[0];
    case miINT16: { int16_t v; memcpy(&v, tmp, 2); return v; }
    case miUINT16: { uint16_t v; memcpy(&v, tmp, 2); return v; }
    case miINT32: { int32_t v; memcpy(&v, tmp, 4); return v; }
    case miUINT32: { uint32_t v; memcpy(&v, tmp, 4); return v; }
    case miSINGLE: { float v; memcpy(&v, tmp, 4); return v; }
    case miDOUBLE: { double v; memcpy(&v, tmp, 8); return v; }
    case miINT64: { int64_t v; memcpy(&v, tmp, 8); return (double)v; }
    case miUINT64: { uint64_t v; memcpy(&v, tmp, 8); return (double)v; }
    default: return 0.0;
    }
}

static int to_double(const mx_t *mx, int swap, double **out, size_t *count)
{
    const int sz = elem_size(mx->re_type);
    if (!sz) return KNN_ERR_FORMAT;
    if (mx->dims[0] < 0 || mx->dims[1] < 0) return KNN_ERR_FORMAT;
    const uint64_t cnt64 = (uint64_t)mx->dims[0] * (uint64_t)mx->dims[1];   /* < 2^62 */
    /* the payload must hold cnt elements: compare by division, no wrap */
    if (cnt64 > (uint64_t)mx->re_bytes / (uint64_t)sz || cnt64 > SIZE_MAX / sizeof(double))
        return KNN_ERR_FORMAT;
    const size_t cnt = (size_t)cnt64;
    double *v = (double *)malloc((cnt ? cnt : 1) * sizeof(double));
    if (!v) return KNN_ERR_NOMEM;
    if (mx->re_type == miDOUBLE && !swap) {
        memcpy(v, mx->re, cnt * sizeof(double));
    } else {
        for (size_t i = 0; i < cnt; i++) v[i] = conv1(mx->re + i * sz, mx->re_type, swap);
    }
    *out = v;
    *count = cnt;
    return KNN_OK;
}

/* Inflate a miCOMPRESSED payload.  With want > 0 only that many output
 * bytes are produced (enough for the tag and the matrix header). */
static int inflate_elem(const uint8_t *src, size_t n, uint8_t **out, size_t *outn, size_t want)
{
    z_stream z;
    memset(&z, 0, sizeof(z));
    if (inflateInit(&z) != Z_OK) return KNN_ERR_FORMAT;
    size_t cap = want ? want : 8;
    uint8_t *buf = (uint8_t *)malloc(cap);
    if (!buf) { inflateEnd(&z); return KNN_ERR_NOMEM; }
    z.next_in = (Bytef *)src;
    z.avail_in = (uInt)(n > 0xffffffffu ? 0xffffffffu : n);
    z.next_out = buf;
    z.avail_out = (uInt)cap;
    int zr = inflate(&z, Z_SYNC_FLUSH);
    size_t got = cap - z.avail_out;
    if (!want) {
        while (zr == Z_OK) {
            if (z.avail_out == 0) {
                size_t ncap = cap * 2;
                uint8_t *nbuf = (uint8_t *)realloc(buf, ncap);
                if (!nbuf) { free(buf); inflateEnd(&z); return KNN_ERR_NOMEM; }
                buf = nbuf;
                z.next_out = buf + cap;
                z.avail_out = (uInt)(ncap - cap);
                cap = ncap;
            }
            zr = inflate(&z, Z_NO_FLUSH);
        }
        if (zr != Z_STREAM_END) { free(buf); inflateEnd(&z); return KNN_ERR_FORMAT; }
        got = cap - z.avail_out;
    } else if (zr != Z_OK && zr != Z_STREAM_END) {
        free(buf);
        inflateEnd(&z);
        return KNN_ERR_FORMAT;
    }
    inflateEnd(&z);
    *out = buf;
    *outn = got;
    return KNN_OK;
}

/* Find variable `name` and convert it; *found set on success. */
static int find_var(const buf_t *file, const char *name, double **vals, size_t *rows, size_t *cols)
{
    size_t off = 128, next;
    uint32_t t, nb;
    const uint8_t *d;
    while (off + 8 <= file->n) {
        if (read_tag(file, off, &t, &nb, &d, &next)) return KNN_ERR_FORMAT;
        mx_t mx;
        if (t == miMATRIX) {
            if (parse_matrix(d, nb, file->swap, &mx, 1) == KNN_OK && strcmp(mx.name, name) == 0) {
                int rc = parse_matrix(d, nb, file->swap, &mx, 0);
                if (rc) return rc;
                size_t cnt;
                rc = to_double(&mx, file->swap, vals, &cnt);
                if (rc) return rc;
                *rows = (size_t)mx.dims[0];
                *cols = (size_t)mx.dims[1];
                return KNN_OK;
            }
        } else if (t == miCOMPRESSED) {
            uint8_t *hdr = NULL;
            size_t hn = 0;
            int rc = inflate_elem(d, nb, &hdr, &hn, 512);
            if (rc) return rc;
            /* the inflated element starts with a miMATRIX tag */
            const int match = hn >= 8 && rd32(hdr, file->swap) == miMATRIX &&
                              parse_matrix(hdr + 8, hn - 8, file->swap, &mx, 1) == KNN_OK &&
                              strcmp(mx.name, name) == 0;
            free(hdr);
            if (match) {
                uint8_t *full = NULL;
                size_t fn = 0;
                rc = inflate_elem(d, nb, &full, &fn, 0);
                if (rc) return rc;
                if (fn < 8 || rd32(full, file->swap) != miMATRIX) { free(full); return KNN_ERR_FORMAT; }
                uint32_t mnb = rd32(full + 4, file->swap);
                if ((size_t)mnb + 8 > fn) { free(full); return KNN_ERR_FORMAT; }
                rc = parse_matrix(full + 8, mnb, file->swap, &mx, 0);
                size_t cnt;
                if (!rc) rc = to_double(&mx, file->swap, vals, &cnt);
                if (!rc) {
                    *rows = (size_t)mx.dims[0];
                    *cols = (size_t)mx.dims[1];
                }
                free(full);
                return rc;
            }
        }
        if (next <= off) break;
        off = next;
    }
    return KNN_ERR_FORMAT;
}

int knn_load_mat(const char *path, const char *xvar, const char *lvar, double **X, size_t *m,
                 size_t *n, double **labels, size_t *nlabels)
{
    if (!path || !xvar || !X || !m || !n) return KNN_ERR_INVALID;
    FILE *f = fopen(path, "rb");
    if (!f) return KNN_ERR_IO;
    if (fseek(f, 0, SEEK_END) != 0) { fclose(f); return KNN_ERR_IO; }
    long sz = ftell(f);
    if (sz < 128) { fclose(f); return KNN_ERR_FORMAT; }
    rewind(f);
    uint8_t *data = (uint8_t *)malloc((size_t)sz);
    if (!data) { fclose(f); return KNN_ERR_NOMEM; }
    if (fread(data, 1, (size_t)sz, f) != (size_t)sz) { free(data); fclose(f); return KNN_ERR_IO; }
    fclose(f);
    int rc = KNN_OK;
    /* v7.3 = HDF5 container: MAT header text, HDF5 superblock at 512 */
    if (memcmp(data, "\x89HDF", 4) == 0 || (sz > 516 && memcmp(data + 512, "\x89HDF", 4) == 0))
        rc = KNN_ERR_UNSUPPORTED;
    buf_t b = {data, (size_t)sz, 0};
    if (!rc) {
        if (data[126] == 'I' && data[127] == 'M') b.swap = 0;
        else if (data[126] == 'M' && data[127] == 'I') b.swap = 1;
        else rc = KNN_ERR_FORMAT;
    }
    double *xv = NULL, *lv = NULL;
    size_t xr = 0, xc = 0, lr = 0, lc = 0;
    if (!rc) rc = find_var(&b, xvar, &xv, &xr, &xc);
    if (!rc && lvar) rc = find_var(&b, lvar, &lv, &lr, &lc);
    free(data);
    if (rc) {
        free(xv);
        free(lv);
        return rc;
    }
    *X = xv;
    *m = xr;
    *n = xc;
    if (labels) *labels = lv;
    else free(lv);
    if (nlabels) *nlabels = lr * lc;
    return KNN_OK;
}
