/*
 * oracle_cli.c -- TEST INFRASTRUCTURE.  Same command line and output files as
 * oracle/ref_harness.c (the reference-driven harness), but driven by the C
 * restatement in hl_oracle.c, so the two can be diffed byte for byte and MB
 * by MB.
 *
 * usage: hlenc_oracle W H N qp me_range deblock gop early_term in.yuv out_prefix [quiet]
 */
#include "hl_oracle.h"
#include "mbrec.h"

#include <stdio.h>
#include <stdlib.h>
#include <time.h>

int main(int argc, char** argv)
{
    hlo_params_t p;
    hlo_enc_t* e;
    const char *in, *pre;
    char path[1024];
    FILE *fi, *fo, *frec = NULL, *fmb = NULL;
    uint8_t *buf, *out;
    int32_t* recs;
    size_t fs, cap, len;
    int N, n = 0, quiet;
    double tot = 0;

    if (argc < 11) {
        fprintf(stderr, "usage: %s W H N qp me_range deblock gop early_term in.yuv out_prefix [quiet]\n", argv[0]);
        return 1;
    }
    p.width = atoi(argv[1]);
    p.height = atoi(argv[2]);
    N = atoi(argv[3]);
    p.qp = atoi(argv[4]);
    p.me_range = atoi(argv[5]);
    p.deblock = atoi(argv[6]);
    p.gop_size = atoi(argv[7]);
    p.early_term = atoi(argv[8]);
    in = argv[9];
    pre = argv[10];
    quiet = argc > 11;
    e = hlo_create(&p);
    if (!e) {
        fprintf(stderr, "bad parameters\n");
        return 2;
    }
    fs = (size_t)p.width * p.height * 3 / 2;
    cap = fs * 2 + (1 << 20);
    buf = (uint8_t*)malloc(fs);
    out = (uint8_t*)malloc(cap);
    recs = (int32_t*)malloc(sizeof(int32_t) * MBR_STRIDE * (size_t)(p.width / 16) * (p.height / 16));
    fi = fopen(in, "rb");
    if (!fi) {
        fprintf(stderr, "cannot open %s\n", in);
        return 3;
    }
    snprintf(path, sizeof(path), "%s.264", pre);
    fo = fopen(path, "wb");
    if (!quiet) {
        snprintf(path, sizeof(path), "%s.rec.yuv", pre);
        frec = fopen(path, "wb");
        snprintf(path, sizeof(path), "%s.mbs", pre);
        fmb = fopen(path, "wb");
    }
    while (n < N && fread(buf, 1, fs, fi) == fs) {
        struct timespec t0, t1;
        const uint8_t* y = buf;
        const uint8_t* u = buf + (size_t)p.width * p.height;
        const uint8_t* v = u + (size_t)p.width * p.height / 4;
        clock_gettime(CLOCK_MONOTONIC, &t0);
        if (hlo_encode_frame(e, y, u, v, out, cap, &len)) {
            fprintf(stderr, "encode error at frame %d\n", n);
            return 4;
        }
        clock_gettime(CLOCK_MONOTONIC, &t1);
        tot += (t1.tv_sec - t0.tv_sec) + (t1.tv_nsec - t0.tv_nsec) * 1e-9;
        fwrite(out, 1, len, fo);
        if (!quiet) {
            fwrite(hlo_recon(e, 0), 1, (size_t)p.width * p.height, frec);
            fwrite(hlo_recon(e, 1), 1, (size_t)p.width * p.height / 4, frec);
            fwrite(hlo_recon(e, 2), 1, (size_t)p.width * p.height / 4, frec);
            hlo_dump_mbs(e, recs);
            fwrite(recs, sizeof(int32_t) * MBR_STRIDE, (size_t)(p.width / 16) * (p.height / 16), fmb);
        }
        n++;
    }
    fclose(fi);
    fclose(fo);
    if (frec) fclose(frec);
    if (fmb) fclose(fmb);
    if (hlo_rdo_overflows(e)) fprintf(stderr, "warning: %lld RDO buffer overflows\n", (long long)hlo_rdo_overflows(e));
    printf("{\"frames\": %d, \"seconds\": %.6f, \"fps\": %.4f, \"mb_per_s\": %.1f}\n", n, tot, n / tot,
           (double)n * (p.width / 16) * (p.height / 16) / tot);
    hlo_destroy(e);
    free(buf);
    free(out);
    free(recs);
    return 0;
}
