/* Compile check only (tests/test_jni_glue.py): the JNI types and the JNIEnv entries
 * jni/deltareplay_jni.c uses, declared from the JNI specification so the glue can be type-checked
 * against include/deltareplay.h in an image without a JDK. Never linked or run; the real build uses
 * the JDK's jni.h (build line in jni/deltareplay_jni.c). Member order is not the JDK's. */
#ifndef DR_JNI_MIN_H
#define DR_JNI_MIN_H
#include <stdint.h>
#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL
#define JNI_ABORT 2
#define JNI_FALSE 0
#define JNI_TRUE 1
typedef int32_t jint;
typedef int64_t jlong;
typedef int8_t jbyte;
typedef uint8_t jboolean;
typedef jint jsize;
typedef struct _jobject* jobject;
typedef jobject jclass, jstring, jthrowable, jarray;
typedef jarray jobjectArray, jbyteArray, jintArray, jlongArray;
typedef struct _jmethodID* jmethodID;
struct JNINativeInterface_;
typedef const struct JNINativeInterface_* JNIEnv;
struct JNINativeInterface_ {
  jclass (*FindClass)(JNIEnv*, const char*);
  jint (*Throw)(JNIEnv*, jthrowable);
  jint (*ThrowNew)(JNIEnv*, jclass, const char*);
  jmethodID (*GetMethodID)(JNIEnv*, jclass, const char*, const char*);
  jobject (*NewObject)(JNIEnv*, jclass, jmethodID, ...);
  jstring (*NewStringUTF)(JNIEnv*, const char*);
  const char* (*GetStringUTFChars)(JNIEnv*, jstring, jboolean*);
  void (*ReleaseStringUTFChars)(JNIEnv*, jstring, const char*);
  jsize (*GetArrayLength)(JNIEnv*, jarray);
  jobjectArray (*NewObjectArray)(JNIEnv*, jsize, jclass, jobject);
  jobject (*GetObjectArrayElement)(JNIEnv*, jobjectArray, jsize);
  void (*SetObjectArrayElement)(JNIEnv*, jobjectArray, jsize, jobject);
  jbyteArray (*NewByteArray)(JNIEnv*, jsize);
  jlongArray (*NewLongArray)(JNIEnv*, jsize);
  jbyte* (*GetByteArrayElements)(JNIEnv*, jbyteArray, jboolean*);
  jint* (*GetIntArrayElements)(JNIEnv*, jintArray, jboolean*);
  jlong* (*GetLongArrayElements)(JNIEnv*, jlongArray, jboolean*);
  void (*ReleaseByteArrayElements)(JNIEnv*, jbyteArray, jbyte*, jint);
  void (*ReleaseIntArrayElements)(JNIEnv*, jintArray, jint*, jint);
  void (*ReleaseLongArrayElements)(JNIEnv*, jlongArray, jlong*, jint);
  void (*GetByteArrayRegion)(JNIEnv*, jbyteArray, jsize, jsize, jbyte*);
  void (*SetByteArrayRegion)(JNIEnv*, jbyteArray, jsize, jsize, const jbyte*);
  void (*SetLongArrayRegion)(JNIEnv*, jlongArray, jsize, jsize, const jlong*);
  jobject (*NewDirectByteBuffer)(JNIEnv*, void*, jlong);
  jboolean (*ExceptionCheck)(JNIEnv*);
  void (*DeleteLocalRef)(JNIEnv*, jobject);
  jint (*EnsureLocalCapacity)(JNIEnv*, jint);
};
#endif
