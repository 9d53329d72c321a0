/*
 * Oracle (TEST INFRASTRUCTURE ONLY -- see svo_oracle.h).
 *
 * Literal restatement of the reference's own bucketing code,
 * R:src/bucket.cpp:24-68 (FeatureSet::bucketingFeatures), :72-101
 * (Bucket::add_feature), :103-106 (Bucket::get_features). Quirks kept:
 *   - (nh+1)*(nw+1) buckets allocated (:36-44) but indexed with stride nw
 *     (:50-53, :62), so cell (r, nw) aliases (r+1, 0) and is read out twice;
 *   - when a bucket is full, the age-min loop (:89-96) compares the incoming
 *     age with age_min and never reads ages[i], so with the all-zero ages of
 *     appendNewFeatures (:18-22) the incoming point always replaces slot 0.
 * This file IS pinned: it restates code that lives in the reference itself.
 */
#include "svo_oracle.h"

#include <stdlib.h>
#include <string.h>

typedef struct {
    int size, max_size;
    float* xy;
    int* ages;
} bucket_t;

static void bucket_add(bucket_t* b, float x, float y, int age)
{
    if (b->size < b->max_size) {
        b->xy[2 * b->size] = x;
        b->xy[2 * b->size + 1] = y;
        b->ages[b->size] = age;
        b->size++;
    } else {
        int age_min = b->ages[0];
        int age_min_idx = 0;
        for (int i = 0; i < b->size; i++) {
            if (age < age_min) {
                age_min = age;
                age_min_idx = i;
            }
        }
        b->xy[2 * age_min_idx] = x;
        b->xy[2 * age_min_idx + 1] = y;
        b->ages[age_min_idx] = age;
    }
}

int svo_oracle_bucket(const float* xy, const int* ages, int n, int img_w, int img_h,
                      int bucket_size, int per_bucket, float* xy_out, int* ages_out,
                      int cap, int* n_total)
{
    int nh = img_h / bucket_size;
    int nw = img_w / bucket_size;
    int nb = (nh + 1) * (nw + 1);
    bucket_t* B = (bucket_t*)calloc((size_t)nb, sizeof(bucket_t));
    float* xy_mem = (float*)malloc(sizeof(float) * 2 * (size_t)nb * (per_bucket > 0 ? per_bucket : 1));
    int* age_mem = (int*)malloc(sizeof(int) * (size_t)nb * (per_bucket > 0 ? per_bucket : 1));
    for (int i = 0; i < nb; i++) {
        B[i].max_size = per_bucket;
        B[i].xy = xy_mem + (size_t)2 * i * per_bucket;
        B[i].ages = age_mem + (size_t)i * per_bucket;
    }
    int ok = 1;
    for (int i = 0; i < n; i++) {
        int hi = (int)(xy[2 * i + 1] / bucket_size);
        int wi = (int)(xy[2 * i] / bucket_size);
        int idx = hi * nw + wi;
        if (idx < 0 || idx >= nb || per_bucket <= 0) { ok = 0; continue; } /* UB in the reference */
        bucket_add(&B[idx], xy[2 * i], xy[2 * i + 1], ages ? ages[i] : 0);
    }
    int count = 0;
    for (int r = 0; r <= nh; r++)
        for (int c = 0; c <= nw; c++) {
            int idx = r * nw + c;
            for (int k = 0; k < B[idx].size; k++) {
                if (count < cap) {
                    xy_out[2 * count] = B[idx].xy[2 * k];
                    xy_out[2 * count + 1] = B[idx].xy[2 * k + 1];
                    if (ages_out) ages_out[count] = B[idx].ages[k];
                }
                count++;
            }
        }
    free(B);
    free(xy_mem);
    free(age_mem);
    if (n_total) *n_total = count;
    (void)ok;
    return count < cap ? count : cap;
}
