/* geohip_jni.c -- the native half of GeoFlink.utils.GeoHip (jvm/src/GeoFlink/utils/GeoHip.java):
 * each native method is one call of the C ABI in include/geohip.h.  Built by jvm/build.sh
 * (gcc -shared against $JAVA_HOME/include and spatialflink_amd/libgeohip.so); source only here,
 * since this image has no JDK.
 *
 * Windows arrive as direct ByteBuffers (GetDirectBufferAddress: no copy, no GC pinning), small
 * arrays (grid, polygon rings, kNN outputs) through Get/Set<Type>ArrayRegion.  Variable-size
 * results use the library's two-phase protocol: a count-only call (cap = 0, GEOHIP_ERR_CAPACITY
 * with the required count), then the call into a buffer of that size.  Status codes become Java
 * exceptions: GEOHIP_ERR_ARG -> IllegalArgumentException (where the reference calls
 * System.exit(1) or throws NumberFormatException), GEOHIP_ERR_UNSUPPORTED ->
 * UnsupportedOperationException, GEOHIP_ERR_OOM -> OutOfMemoryError, otherwise
 * RuntimeException; the message is geohip_last_error. */
#include <jni.h>
#include <stdint.h>
#include <stdlib.h>

#include "geohip.h"

#define CTX(h) ((geohip_ctx*)(intptr_t)(h))

static void throw_msg(JNIEnv* env, const char* cls, const char* msg) {
    jclass c = (*env)->FindClass(env, cls);
    if (c) (*env)->ThrowNew(env, c, msg);
}

static void throw_for(JNIEnv* env, geohip_ctx* ctx, int rc) {
    const char* cls = rc == GEOHIP_ERR_ARG           ? "java/lang/IllegalArgumentException"
                      : rc == GEOHIP_ERR_UNSUPPORTED ? "java/lang/UnsupportedOperationException"
                      : rc == GEOHIP_ERR_OOM         ? "java/lang/OutOfMemoryError"
                                                     : "java/lang/RuntimeException";
    throw_msg(env, cls, ctx ? geohip_last_error(ctx) : "libgeohip error");
}

static geohip_grid grid_of(JNIEnv* env, jdoubleArray g) {
    jdouble v[4] = {0, 0, 0, 0};
    (*env)->GetDoubleArrayRegion(env, g, 0, 4, v);
    geohip_grid r = {v[0], v[1], v[2], (int32_t)v[3], 0};
    return r;
}

/* The n doubles of a direct ByteBuffer, or NULL when b is null, not direct (a heap buffer has no
 * address) or smaller than 8 * n bytes: the library would read past it. */
static const double* dbuf(JNIEnv* env, jobject b, jlong n) {
    if (!b || n < 0) return NULL;
    void* p = (*env)->GetDirectBufferAddress(env, b);
    if (!p || (*env)->GetDirectBufferCapacity(env, b) < 8 * n) return NULL;
    return (const double*)p;
}

/* x / y of an n-point window; throws IllegalArgumentException and returns 0 when either is unusable */
static int window_bufs(JNIEnv* env, jobject x, jobject y, jint n, const double** px, const double** py) {
    *px = dbuf(env, x, n);
    *py = dbuf(env, y, n);
    if (n < 0 || !*px || !*py) {
        throw_msg(env, "java/lang/IllegalArgumentException",
                  "coordinates must be direct ByteBuffers of at least 8 * n bytes (n >= 0)");
        return 0;
    }
    return 1;
}

/* a caller-supplied output array of at least len elements (kNN results) */
static int out_len_ok(JNIEnv* env, jarray a, jint len) {
    if (a && (*env)->GetArrayLength(env, a) >= len) return 1;
    throw_msg(env, "java/lang/IllegalArgumentException", "kNN output arrays must hold k elements");
    return 0;
}

static void throw_oom(JNIEnv* env, const char* what) { throw_msg(env, "java/lang/OutOfMemoryError", what); }

/* a Java int[] as a malloc'd uint32_t copy (NULL for a null array); *len its length */
static uint32_t* u32_copy(JNIEnv* env, jintArray a, jsize* len) {
    *len = 0;
    if (!a) return NULL;
    *len = (*env)->GetArrayLength(env, a);
    uint32_t* p = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)(*len ? *len : 1));
    if (p && *len) (*env)->GetIntArrayRegion(env, a, 0, *len, (jint*)p);
    return p;
}

static double* f64_copy(JNIEnv* env, jdoubleArray a, jsize* len) {
    *len = a ? (*env)->GetArrayLength(env, a) : 0;
    double* p = (double*)malloc(sizeof(double) * (size_t)(*len ? *len : 1));
    if (p && *len) (*env)->GetDoubleArrayRegion(env, a, 0, *len, p);
    return p;
}

/* m pairs (2 * m uint32) as a flat Java int[] (NULL and an exception when it cannot hold them) */
static jintArray pairs_array(JNIEnv* env, const uint32_t* pairs, uint64_t m) {
    if (2 * m > 0x7fffffffull) {
        throw_msg(env, "java/lang/UnsupportedOperationException", "more pairs than a Java int[] holds");
        return NULL;
    }
    jintArray res = (*env)->NewIntArray(env, (jsize)(2 * m));
    if (res && m) (*env)->SetIntArrayRegion(env, res, 0, (jsize)(2 * m), (const jint*)pairs);
    return res;
}

JNIEXPORT jint JNICALL Java_GeoFlink_utils_GeoHip_abiVersion(JNIEnv* env, jclass c) { return geohip_abi_version(); }

JNIEXPORT jlong JNICALL Java_GeoFlink_utils_GeoHip_create(JNIEnv* env, jclass c, jint mask) {
    geohip_ctx* ctx = NULL;
    int rc = geohip_ctx_create((uint32_t)mask, &ctx);
    if (rc) throw_for(env, NULL, rc);
    return (jlong)(intptr_t)ctx;
}

JNIEXPORT void JNICALL Java_GeoFlink_utils_GeoHip_destroy(JNIEnv* env, jclass c, jlong h) { geohip_ctx_destroy(CTX(h)); }

JNIEXPORT void JNICALL Java_GeoFlink_utils_GeoHip_rangeOrder(JNIEnv* env, jclass c, jlong h, jint order) {
    int rc = geohip_ctx_set_range_order(CTX(h), (int)order);
    if (rc) throw_for(env, CTX(h), rc);
}

JNIEXPORT jintArray JNICALL Java_GeoFlink_utils_GeoHip_rangePP(JNIEnv* env, jclass c, jlong h, jdoubleArray g, jobject x,
                                                               jobject y, jint n, jdouble qx, jdouble qy, jdouble r,
                                                               jboolean approx) {
    geohip_grid grid = grid_of(env, g);
    const double *px, *py;
    if (!window_bufs(env, x, y, n, &px, &py)) return NULL;
    uint32_t* out = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)(n > 0 ? n : 1));  /* hits <= n */
    if (!out) {
        throw_oom(env, "range hit buffer");
        return NULL;
    }
    uint64_t cnt = 0;
    int rc = geohip_range_pp(CTX(h), &grid, px, py, (uint64_t)n, qx, qy, r, approx, out, (uint64_t)n, &cnt);
    jintArray res = NULL;
    if (rc) {
        throw_for(env, CTX(h), rc);
    } else {
        res = (*env)->NewIntArray(env, (jsize)cnt);
        if (res && cnt) (*env)->SetIntArrayRegion(env, res, 0, (jsize)cnt, (const jint*)out);
    }
    free(out);
    return res;
}

JNIEXPORT jint JNICALL Java_GeoFlink_utils_GeoHip_knnPP(JNIEnv* env, jclass c, jlong h, jdoubleArray g, jobject x,
                                                        jobject y, jint n, jdouble qx, jdouble qy, jdouble r, jint k,
                                                        jintArray oi, jdoubleArray od) {
    geohip_grid grid = grid_of(env, g);
    const double *px, *py;
    if (!window_bufs(env, x, y, n, &px, &py) || !out_len_ok(env, oi, k) || !out_len_ok(env, od, k)) return -1;
    uint32_t* idx = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)(k > 0 ? k : 1));
    double* dist = (double*)malloc(sizeof(double) * (size_t)(k > 0 ? k : 1));
    if (!idx || !dist) {
        free(idx);
        free(dist);
        throw_oom(env, "kNN result buffer");
        return -1;
    }
    uint32_t cnt = 0;
    int rc = geohip_knn_pp(CTX(h), &grid, px, py, (uint64_t)n, qx, qy, r, (uint32_t)k, idx, dist, &cnt);
    if (!rc && cnt) {
        (*env)->SetIntArrayRegion(env, oi, 0, (jsize)cnt, (const jint*)idx);
        (*env)->SetDoubleArrayRegion(env, od, 0, (jsize)cnt, dist);
    }
    free(idx);
    free(dist);
    if (rc) {
        throw_for(env, CTX(h), rc);
        return -1;
    }
    return (jint)cnt;
}

JNIEXPORT jobjectArray JNICALL Java_GeoFlink_utils_GeoHip_knnRangePP(JNIEnv* env, jclass c, jlong h, jdoubleArray g,
                                                                      jobject x, jobject y, jint n, jdouble qx,
                                                                      jdouble qy, jdouble r, jint k, jboolean approx,
                                                                      jintArray ki, jdoubleArray kd) {
    geohip_grid grid = grid_of(env, g);
    const double *px, *py;
    if (!window_bufs(env, x, y, n, &px, &py) || !out_len_ok(env, ki, k) || !out_len_ok(env, kd, k)) return NULL;
    uint32_t* idx = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)(k > 0 ? k : 1));
    double* dist = (double*)malloc(sizeof(double) * (size_t)(k > 0 ? k : 1));
    uint32_t* hits = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)(n > 0 ? n : 1));
    if (!idx || !dist || !hits) {
        free(idx);
        free(dist);
        free(hits);
        throw_oom(env, "kNN + range result buffers");
        return NULL;
    }
    uint32_t kcnt = 0;
    uint64_t rcnt = 0;
    int rc = geohip_knn_range_pp(CTX(h), &grid, px, py, (uint64_t)n, qx, qy, r, (uint32_t)k, approx, idx, dist, &kcnt,
                                 hits, (uint64_t)n, &rcnt);
    jobjectArray res = NULL;
    if (rc) {
        throw_for(env, CTX(h), rc);
    } else {
        if (kcnt) {
            (*env)->SetIntArrayRegion(env, ki, 0, (jsize)kcnt, (const jint*)idx);
            (*env)->SetDoubleArrayRegion(env, kd, 0, (jsize)kcnt, dist);
        }
        jintArray count = (*env)->NewIntArray(env, 1);
        jint kc = (jint)kcnt;
        jintArray range = (*env)->NewIntArray(env, (jsize)rcnt);
        if (count && range) {
            (*env)->SetIntArrayRegion(env, count, 0, 1, &kc);
            if (rcnt) (*env)->SetIntArrayRegion(env, range, 0, (jsize)rcnt, (const jint*)hits);
            res = (*env)->NewObjectArray(env, 2, (*env)->GetObjectClass(env, count), NULL);
            if (res) {
                (*env)->SetObjectArrayElement(env, res, 0, count);
                (*env)->SetObjectArrayElement(env, res, 1, range);
            }
        }
    }
    free(idx);
    free(dist);
    free(hits);
    return res;
}

JNIEXPORT jintArray JNICALL Java_GeoFlink_utils_GeoHip_joinPP(JNIEnv* env, jclass c, jlong h, jdoubleArray gd,
                                                              jdoubleArray gq, jobject dx, jobject dy, jint nd,
                                                              jobject qx, jobject qy, jint nq, jdouble r,
                                                              jboolean approx) {
    geohip_grid a = grid_of(env, gd), b = grid_of(env, gq);
    const double *px, *py, *ox, *oy;
    if (!window_bufs(env, dx, dy, nd, &px, &py) || !window_bufs(env, qx, qy, nq, &ox, &oy)) return NULL;
    uint64_t cnt = 0;
    int rc = geohip_join_pp_count_only(CTX(h), &a, &b, px, py, (uint64_t)nd, ox, oy, (uint64_t)nq, r, approx, &cnt);
    if (rc) {
        throw_for(env, CTX(h), rc);
        return NULL;
    }
    uint32_t* pairs = (uint32_t*)malloc(sizeof(uint32_t) * 2 * (size_t)(cnt ? cnt : 1));
    if (!pairs) {
        throw_oom(env, "join pair buffer");
        return NULL;
    }
    uint64_t m = 0;
    rc = geohip_join_pp(CTX(h), &a, &b, px, py, (uint64_t)nd, ox, oy, (uint64_t)nq, r, approx, pairs, cnt, &m);
    jintArray res = NULL;
    if (rc) throw_for(env, CTX(h), rc);
    else res = pairs_array(env, pairs, m);
    free(pairs);
    return res;
}

typedef int (*ppoly_fn)(geohip_ctx*, const geohip_grid*, const geohip_grid*, const double*, const double*, uint64_t,
                        const uint32_t*, const uint32_t*, const double*, const double*, uint64_t, uint32_t, double, int,
                        uint32_t*, uint64_t, uint64_t*);

static int range_ppoly_2g(geohip_ctx* ctx, const geohip_grid* g, const geohip_grid* unused, const double* x,
                          const double* y, uint64_t n, const uint32_t* pr, const uint32_t* ro, const double* vx,
                          const double* vy, uint64_t nv, uint32_t np, double r, int a, uint32_t* out, uint64_t cap,
                          uint64_t* cnt) {
    (void)unused;
    return geohip_range_ppoly(ctx, g, x, y, n, pr, ro, vx, vy, nv, np, r, a, out, cap, cnt);
}

/* both point-polygon pair calls, two-phase */
static jintArray ppoly_pairs(JNIEnv* env, jlong h, ppoly_fn fn, jdoubleArray g1, jdoubleArray g2, jobject x, jobject y,
                             jint n, jintArray polyRings, jintArray ringOff, jdoubleArray vx, jdoubleArray vy,
                             jdouble r, jboolean approx) {
    geohip_grid a = grid_of(env, g1), b = grid_of(env, g2 ? g2 : g1);
    const double *px, *py;
    if (!window_bufs(env, x, y, n, &px, &py)) return NULL;
    jsize npr = 0, nro = 0, nvx = 0, nvy = 0;
    uint32_t* pr = u32_copy(env, polyRings, &npr);
    uint32_t* ro = u32_copy(env, ringOff, &nro);
    double* hx = f64_copy(env, vx, &nvx);
    double* hy = f64_copy(env, vy, &nvy);
    jintArray res = NULL;
    const uint32_t npoly = pr ? (npr > 0 ? (uint32_t)(npr - 1) : 0u) : (nro > 0 ? (uint32_t)(nro - 1) : 0u);
    if (!ro || !hx || !hy || nvx != nvy) {
        throw_msg(env, "java/lang/IllegalArgumentException", "polygon arrays");
    } else {
        uint64_t cnt = 0;
        int rc = fn(CTX(h), &a, &b, px, py, (uint64_t)n, pr, ro, hx, hy, (uint64_t)nvx, npoly, r, approx, NULL, 0,
                    &cnt);
        if (rc && rc != GEOHIP_ERR_CAPACITY) {
            throw_for(env, CTX(h), rc);
        } else {
            uint32_t* pairs = (uint32_t*)malloc(sizeof(uint32_t) * 2 * (size_t)(cnt ? cnt : 1));
            uint64_t m = 0;
            rc = pairs ? fn(CTX(h), &a, &b, px, py, (uint64_t)n, pr, ro, hx, hy, (uint64_t)nvx, npoly, r, approx, pairs,
                            cnt, &m)
                       : GEOHIP_ERR_OOM;
            if (!pairs) throw_oom(env, "point-polygon pair buffer");
            else if (rc) throw_for(env, CTX(h), rc);
            else res = pairs_array(env, pairs, m);
            free(pairs);
        }
    }
    free(pr);
    free(ro);
    free(hx);
    free(hy);
    return res;
}

JNIEXPORT jintArray JNICALL Java_GeoFlink_utils_GeoHip_rangePPoly(JNIEnv* env, jclass c, jlong h, jdoubleArray g,
                                                                  jobject x, jobject y, jint n, jintArray polyRings,
                                                                  jintArray ringOff, jdoubleArray vx, jdoubleArray vy,
                                                                  jdouble r, jboolean approx) {
    return ppoly_pairs(env, h, range_ppoly_2g, g, NULL, x, y, n, polyRings, ringOff, vx, vy, r, approx);
}

JNIEXPORT jintArray JNICALL Java_GeoFlink_utils_GeoHip_joinPPoly(JNIEnv* env, jclass c, jlong h, jdoubleArray gu,
                                                                 jdoubleArray gq, jobject x, jobject y, jint n,
                                                                 jintArray polyRings, jintArray ringOff,
                                                                 jdoubleArray vx, jdoubleArray vy, jdouble r,
                                                                 jboolean approx) {
    return ppoly_pairs(env, h, geohip_join_ppoly, gu, gq, x, y, n, polyRings, ringOff, vx, vy, r, approx);
}

JNIEXPORT jint JNICALL Java_GeoFlink_utils_GeoHip_knnPPoly(JNIEnv* env, jclass c, jlong h, jdoubleArray g, jobject x,
                                                           jobject y, jint n, jintArray ringOff, jdoubleArray vx,
                                                           jdoubleArray vy, jdouble r, jint k, jboolean approx,
                                                           jintArray oi, jdoubleArray od) {
    geohip_grid grid = grid_of(env, g);
    const double *px, *py;
    if (!window_bufs(env, x, y, n, &px, &py) || !out_len_ok(env, oi, k) || !out_len_ok(env, od, k)) return -1;
    jsize nro = 0, nvx = 0, nvy = 0;
    uint32_t* ro = u32_copy(env, ringOff, &nro);
    double* hx = f64_copy(env, vx, &nvx);
    double* hy = f64_copy(env, vy, &nvy);
    uint32_t* idx = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)(k > 0 ? k : 1));
    double* dist = (double*)malloc(sizeof(double) * (size_t)(k > 0 ? k : 1));
    uint32_t cnt = 0;
    const int oom = !idx || !dist;
    const int bad = !ro || !hx || !hy || nro < 2 || nvx != nvy;
    int rc = oom ? GEOHIP_ERR_OOM
                 : bad ? GEOHIP_ERR_ARG
                       : geohip_knn_ppoly(CTX(h), &grid, px, py, (uint64_t)n, ro, (uint32_t)(nro - 1), hx, hy,
                                          (uint64_t)nvx, r, (uint32_t)k, approx, idx, dist, &cnt);
    if (!rc && cnt) {
        (*env)->SetIntArrayRegion(env, oi, 0, (jsize)cnt, (const jint*)idx);
        (*env)->SetDoubleArrayRegion(env, od, 0, (jsize)cnt, dist);
    }
    free(ro);
    free(hx);
    free(hy);
    free(idx);
    free(dist);
    if (rc) {
        if (oom) throw_oom(env, "kNN result buffer");
        else if (bad) throw_msg(env, "java/lang/IllegalArgumentException", "polygon arrays");
        else throw_for(env, CTX(h), rc);
        return -1;
    }
    return (jint)cnt;
}
