/* Test-only stand-in for a JDK's jni.h (this image has no JDK): the JNI primitive types, handles
 * and the JNINativeInterface members jvm/native/geohip_jni.c calls, with the JNI specification's
 * signatures.  Member ORDER is not the JDK's -- the shim uses members by name, and this header is
 * only ever compiled with tests/jni_stub/fake_jni.c, whose function table fills them.  A real build
 * (jvm/build.sh) uses $JAVA_HOME/include/jni.h. */
#ifndef GEOHIP_TEST_JNI_H
#define GEOHIP_TEST_JNI_H
#include <stdint.h>

#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL

typedef int32_t jint;
typedef int64_t jlong;
typedef int8_t jbyte;
typedef uint8_t jboolean;
typedef uint16_t jchar;
typedef int16_t jshort;
typedef float jfloat;
typedef double jdouble;
typedef jint jsize;

struct _jobject;
typedef struct _jobject* jobject;
typedef jobject jclass;
typedef jobject jthrowable;
typedef jobject jstring;
typedef jobject jarray;
typedef jarray jintArray;
typedef jarray jdoubleArray;
typedef jarray jobjectArray;

struct JNINativeInterface_;
typedef const struct JNINativeInterface_* JNIEnv;

struct JNINativeInterface_ {
    jclass (JNICALL* FindClass)(JNIEnv* env, const char* name);
    jint (JNICALL* ThrowNew)(JNIEnv* env, jclass clazz, const char* msg);
    jclass (JNICALL* GetObjectClass)(JNIEnv* env, jobject obj);
    jsize (JNICALL* GetArrayLength)(JNIEnv* env, jarray array);
    jobjectArray (JNICALL* NewObjectArray)(JNIEnv* env, jsize len, jclass clazz, jobject init);
    void (JNICALL* SetObjectArrayElement)(JNIEnv* env, jobjectArray array, jsize index, jobject val);
    jintArray (JNICALL* NewIntArray)(JNIEnv* env, jsize len);
    void (JNICALL* GetIntArrayRegion)(JNIEnv* env, jintArray array, jsize start, jsize len, jint* buf);
    void (JNICALL* GetDoubleArrayRegion)(JNIEnv* env, jdoubleArray array, jsize start, jsize len, jdouble* buf);
    void (JNICALL* SetIntArrayRegion)(JNIEnv* env, jintArray array, jsize start, jsize len, const jint* buf);
    void (JNICALL* SetDoubleArrayRegion)(JNIEnv* env, jdoubleArray array, jsize start, jsize len, const jdouble* buf);
    void* (JNICALL* GetDirectBufferAddress)(JNIEnv* env, jobject buf);
    jlong (JNICALL* GetDirectBufferCapacity)(JNIEnv* env, jobject buf);
};

#endif
