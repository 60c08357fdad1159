/*!
 * \file dmlc/endian.h
 * \brief Endianness detection.  Parity: reference `include/dmlc/endian.h:9-15`.
 *  MI355X hosts (x86-64) and the GPU are little-endian; the serializer writes
 *  native byte order (see serializer.h), so the macro is informational.
 */
#ifndef DMLC_ENDIAN_H_
#define DMLC_ENDIAN_H_

#define DMLC_LITTLE_ENDIAN (__BYTE_ORDER__ == __ORDER_LITTLE_ENDIAN__)
#define DMLC_IO_NO_ENDIAN_SWAP 1

#endif  // DMLC_ENDIAN_H_
