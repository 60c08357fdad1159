/*!
 * \file src/python/dlpack.h
 * \brief Minimal DLPack ABI (v0.8 layout) for zero-copy hand-off of HBM CSR
 *  arrays to PyTorch (`torch.from_dlpack`).  Device type 10 = kDLROCM.
 */
#ifndef DMLC_PYTHON_DLPACK_H_
#define DMLC_PYTHON_DLPACK_H_

#include <cstdint>

extern "C" {
typedef enum { kDLCPU = 1, kDLROCM = 10 } DLDeviceType;
typedef struct {
  int32_t device_type;
  int32_t device_id;
} DLDevice;
typedef enum { kDLInt = 0U, kDLUInt = 1U, kDLFloat = 2U } DLDataTypeCode;
typedef struct {
  uint8_t code;
  uint8_t bits;
  uint16_t lanes;
} DLDataType;
typedef struct {
  void* data;
  DLDevice device;
  int32_t ndim;
  DLDataType dtype;
  int64_t* shape;
  int64_t* strides;
  uint64_t byte_offset;
} DLTensor;
typedef struct DLManagedTensor {
  DLTensor dl_tensor;
  void* manager_ctx;
  void (*deleter)(struct DLManagedTensor* self);
} DLManagedTensor;
}

#endif  // DMLC_PYTHON_DLPACK_H_
