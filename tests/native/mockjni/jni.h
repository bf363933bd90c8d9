/*
 * TEST DOUBLE of the subset of the JNI C interface that jni/ozec_jni.c uses -- NOT the JDK's jni.h (no JDK exists in
 * this image).  Same type and function names, so jni/ozec_jni.c compiles unchanged against it, but the function
 * table layout differs from a real JVM's: the library built with it only ever runs under tests/native/mockjni/
 * mockjni.c, which implements these functions over fake Java objects so the glue's logic (null slots, offsets,
 * pinning and unpinning, exception selection) is tested on CPU and, for the compute calls, on the GPU.
 */
#ifndef MOCK_JNI_H
#define MOCK_JNI_H
#include <stdint.h>

#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL
#define JNI_ABORT 2
#define JNI_VERSION_1_8 0x00010008

typedef int32_t jint;
typedef int64_t jlong;
typedef int8_t jbyte;
typedef uint8_t jboolean;
typedef jint jsize;

struct mock_object;
typedef struct mock_object *jobject;
typedef jobject jclass;
typedef jobject jarray;
typedef jarray jobjectArray;
typedef jarray jintArray;
typedef jarray jbyteArray;
typedef struct JavaVM_ *JavaVM;

struct JNINativeInterface_;
typedef const struct JNINativeInterface_ *JNIEnv;

struct JNINativeInterface_ {
  jclass (*FindClass)(JNIEnv *, const char *);
  jint (*ThrowNew)(JNIEnv *, jclass, const char *);
  void (*ExceptionClear)(JNIEnv *);
  void (*DeleteLocalRef)(JNIEnv *, jobject);
  jsize (*GetArrayLength)(JNIEnv *, jarray);
  jobject (*GetObjectArrayElement)(JNIEnv *, jobjectArray, jsize);
  void (*GetIntArrayRegion)(JNIEnv *, jintArray, jsize, jsize, jint *);
  void *(*GetPrimitiveArrayCritical)(JNIEnv *, jarray, jboolean *);
  void (*ReleasePrimitiveArrayCritical)(JNIEnv *, jarray, void *, jint);
  jobject (*NewDirectByteBuffer)(JNIEnv *, void *, jlong);
  void *(*GetDirectBufferAddress)(JNIEnv *, jobject);
  jlong (*GetDirectBufferCapacity)(JNIEnv *, jobject);
  void (*GetByteArrayRegion)(JNIEnv *, jbyteArray, jsize, jsize, jbyte *);
  void (*SetByteArrayRegion)(JNIEnv *, jbyteArray, jsize, jsize, const jbyte *);
  jintArray (*NewIntArray)(JNIEnv *, jsize);
  void (*SetIntArrayRegion)(JNIEnv *, jintArray, jsize, jsize, const jint *);
  jboolean (*ExceptionCheck)(JNIEnv *);
};
#endif
