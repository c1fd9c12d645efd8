/* A fake JNIEnv for driving jvm/native/geohip_jni.c without a JVM (test infrastructure).
 *
 * Java objects are heap records: direct ByteBuffers (address + capacity in bytes; a NULL address
 * stands for a heap buffer, which JNI reports as having none), int[] / double[] / Object[] arrays
 * and classes (by name).  ThrowNew records the pending exception's class and message; region
 * accesses outside an array raise ArrayIndexOutOfBoundsException as the JVM does.  The test
 * (tests/test_jni_harness.py) builds objects with the fake_* functions over ctypes, calls the
 * shim's Java_GeoFlink_utils_GeoHip_* entry points with fake_env(), and reads results back. */
#include <stdlib.h>
#include <string.h>

#include "jni.h"

enum { K_DIRECT, K_INTS, K_DOUBLES, K_OBJECTS, K_CLASS };

struct _jobject {
    int kind;
    jsize len;      /* arrays */
    void* data;     /* arrays (owned) / direct buffers (borrowed) */
    jlong cap;      /* direct buffers: bytes */
    char cls[96];   /* classes, and the element class of an Object[] */
    struct _jobject* next;
};

static struct _jobject* all_objects;
static char exc_cls[96], exc_msg[512];

static jobject new_obj(int kind) {
    struct _jobject* o = (struct _jobject*)calloc(1, sizeof(*o));
    if (!o) abort();
    o->kind = kind;
    o->next = all_objects;
    all_objects = o;
    return o;
}

static void raise_exc(const char* cls, const char* msg) {
    if (exc_cls[0]) return;  /* the first pending exception wins */
    strncpy(exc_cls, cls, sizeof(exc_cls) - 1);
    strncpy(exc_msg, msg ? msg : "", sizeof(exc_msg) - 1);
}

static int in_range(jarray a, jsize start, jsize len) {
    if (a && start >= 0 && len >= 0 && (long long)start + len <= a->len) return 1;
    raise_exc(a ? "java/lang/ArrayIndexOutOfBoundsException" : "java/lang/NullPointerException", "region");
    return 0;
}

static jobject new_array(int kind, jsize len, size_t esz) {
    jobject a = new_obj(kind);
    a->len = len;
    a->data = calloc(len > 0 ? (size_t)len : 1, esz);
    if (!a->data) abort();
    return a;
}

static jclass JNICALL f_FindClass(JNIEnv* env, const char* name) {
    (void)env;
    jobject c = new_obj(K_CLASS);
    strncpy(c->cls, name, sizeof(c->cls) - 1);
    return c;
}
static jint JNICALL f_ThrowNew(JNIEnv* env, jclass c, const char* msg) {
    (void)env;
    raise_exc(c ? c->cls : "?", msg);
    return 0;
}
static jclass JNICALL f_GetObjectClass(JNIEnv* env, jobject o) {
    return f_FindClass(env, !o ? "null" : o->kind == K_INTS ? "[I" : o->kind == K_DOUBLES ? "[D" : "java/lang/Object");
}
static jsize JNICALL f_GetArrayLength(JNIEnv* env, jarray a) {
    (void)env;
    if (!a) raise_exc("java/lang/NullPointerException", "array");
    return a ? a->len : 0;
}
static jobjectArray JNICALL f_NewObjectArray(JNIEnv* env, jsize len, jclass c, jobject init) {
    (void)env;
    jobject a = new_array(K_OBJECTS, len, sizeof(jobject));
    if (c) strncpy(a->cls, c->cls, sizeof(a->cls) - 1);
    for (jsize i = 0; i < len; i++) ((jobject*)a->data)[i] = init;
    return a;
}
static void JNICALL f_SetObjectArrayElement(JNIEnv* env, jobjectArray a, jsize i, jobject v) {
    (void)env;
    if (in_range(a, i, 1)) ((jobject*)a->data)[i] = v;
}
static jintArray JNICALL f_NewIntArray(JNIEnv* env, jsize len) {
    (void)env;
    if (len < 0) {
        raise_exc("java/lang/NegativeArraySizeException", "NewIntArray");
        return NULL;
    }
    return new_array(K_INTS, len, sizeof(jint));
}
static void JNICALL f_GetIntArrayRegion(JNIEnv* env, jintArray a, jsize s, jsize n, jint* buf) {
    (void)env;
    if (in_range(a, s, n)) memcpy(buf, (jint*)a->data + s, sizeof(jint) * (size_t)n);
}
static void JNICALL f_GetDoubleArrayRegion(JNIEnv* env, jdoubleArray a, jsize s, jsize n, jdouble* buf) {
    (void)env;
    if (in_range(a, s, n)) memcpy(buf, (jdouble*)a->data + s, sizeof(jdouble) * (size_t)n);
}
static void JNICALL f_SetIntArrayRegion(JNIEnv* env, jintArray a, jsize s, jsize n, const jint* buf) {
    (void)env;
    if (in_range(a, s, n)) memcpy((jint*)a->data + s, buf, sizeof(jint) * (size_t)n);
}
static void JNICALL f_SetDoubleArrayRegion(JNIEnv* env, jdoubleArray a, jsize s, jsize n, const jdouble* buf) {
    (void)env;
    if (in_range(a, s, n)) memcpy((jdouble*)a->data + s, buf, sizeof(jdouble) * (size_t)n);
}
static void* JNICALL f_GetDirectBufferAddress(JNIEnv* env, jobject b) {
    (void)env;
    return b && b->kind == K_DIRECT ? b->data : NULL;
}
static jlong JNICALL f_GetDirectBufferCapacity(JNIEnv* env, jobject b) {
    (void)env;
    return b && b->kind == K_DIRECT && b->data ? b->cap : -1;
}

static const struct JNINativeInterface_ table = {
    f_FindClass,          f_ThrowNew,           f_GetObjectClass,        f_GetArrayLength,
    f_NewObjectArray,     f_SetObjectArrayElement, f_NewIntArray,       f_GetIntArrayRegion,
    f_GetDoubleArrayRegion, f_SetIntArrayRegion, f_SetDoubleArrayRegion, f_GetDirectBufferAddress,
    f_GetDirectBufferCapacity,
};
static JNIEnv the_env = &table;

/* ---- the test's side (ctypes) */
JNIEnv* fake_env(void) { return &the_env; }

/* a direct ByteBuffer over p (cap bytes); p == NULL: a heap buffer (no address) */
jobject fake_direct(void* p, jlong cap) {
    jobject b = new_obj(K_DIRECT);
    b->data = p;
    b->cap = cap;
    return b;
}

jobject fake_ints(const jint* init, jsize len) {
    jobject a = new_array(K_INTS, len, sizeof(jint));
    if (init && len > 0) memcpy(a->data, init, sizeof(jint) * (size_t)len);
    return a;
}

jobject fake_doubles(const jdouble* init, jsize len) {
    jobject a = new_array(K_DOUBLES, len, sizeof(jdouble));
    if (init && len > 0) memcpy(a->data, init, sizeof(jdouble) * (size_t)len);
    return a;
}

jsize fake_len(jobject a) { return a ? a->len : -1; }
void* fake_data(jobject a) { return a ? a->data : NULL; }
jobject fake_elem(jobject a, jsize i) { return a && a->kind == K_OBJECTS && i >= 0 && i < a->len ? ((jobject*)a->data)[i] : NULL; }
const char* fake_exception_class(void) { return exc_cls; }
const char* fake_exception_message(void) { return exc_msg; }
void fake_clear(void) { exc_cls[0] = exc_msg[0] = 0; }

/* free every object made since the last reset (direct buffers' memory belongs to the test) */
void fake_reset(void) {
    while (all_objects) {
        struct _jobject* o = all_objects;
        all_objects = o->next;
        if (o->kind != K_DIRECT) free(o->data);
        free(o);
    }
    fake_clear();
}
