/* Declaration-only stand-in for the JDK's jni.h (TEST INFRASTRUCTURE).
 * Lets tests/test_bindings_cpu.py compile and link the reference JNI source
 * (src/jni/org_janelia_simview_lfm_LFMJNI.cpp) against include/lfm and
 * liblfm.so to prove source/link compatibility of the C ABI; never executed. */
#ifndef LFM_TEST_JNI_SHIM_H
#define LFM_TEST_JNI_SHIM_H
#include <stdint.h>
typedef int32_t jint;
typedef int64_t jlong;
typedef int8_t jbyte;
typedef uint8_t jboolean;
typedef uint16_t jchar;
typedef int16_t jshort;
typedef float jfloat;
typedef double jdouble;
typedef jint jsize;
class _jobject {};
typedef _jobject* jobject;
typedef jobject jclass;
typedef jobject jstring;
typedef jobject jarray;
typedef jarray jbooleanArray;
typedef jarray jbyteArray;
typedef jarray jcharArray;
typedef jarray jshortArray;
typedef jarray jintArray;
typedef jarray jlongArray;
typedef jarray jfloatArray;
typedef jarray jdoubleArray;
#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL
#define JNI_FALSE 0
#define JNI_TRUE 1
#define JNI_COMMIT 1
#define JNI_ABORT 2
struct JNIEnv {
    const char* GetStringUTFChars(jstring, jboolean*);
    void ReleaseStringUTFChars(jstring, const char*);
    jbyte* GetByteArrayElements(jbyteArray, jboolean*);
    void ReleaseByteArrayElements(jbyteArray, jbyte*, jint);
    jshort* GetShortArrayElements(jshortArray, jboolean*);
    void ReleaseShortArrayElements(jshortArray, jshort*, jint);
    jint* GetIntArrayElements(jintArray, jboolean*);
    void ReleaseIntArrayElements(jintArray, jint*, jint);
    jlong* GetLongArrayElements(jlongArray, jboolean*);
    void ReleaseLongArrayElements(jlongArray, jlong*, jint);
    jfloat* GetFloatArrayElements(jfloatArray, jboolean*);
    void ReleaseFloatArrayElements(jfloatArray, jfloat*, jint);
    jdouble* GetDoubleArrayElements(jdoubleArray, jboolean*);
    void ReleaseDoubleArrayElements(jdoubleArray, jdouble*, jint);
    void* GetDirectBufferAddress(jobject);
};
#endif
