// Decoding of libyara regexp programs (the byte code re.c emits and runs).
//
// Opcodes and operand layouts: libyara/include/yara/re.h:65-92 and re.c:65-87
// (RE_SPLIT_ID_TYPE = uint8_t; RE_REPEAT_ARGS = {u16 min, u16 max, i32 offset}
// and RE_REPEAT_ANY_ARGS = {u16 min, u16 max}, both packed; RE_CLASS =
// {u8 negated, u8 bitmap[32]}, types.h:382-386).  Jump and split offsets are
// relative to the instruction's own address.  Host and device share this
// header; the product validates every program it uploads with it.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace yamd {

enum ReOp : uint8_t {
  kOpAny = 0xA0, kOpLiteral = 0xA2, kOpMaskedLiteral = 0xA4, kOpClass = 0xA5,
  kOpWordChar = 0xA7, kOpNonWordChar = 0xA8, kOpSpace = 0xA9, kOpNonSpace = 0xAA,
  kOpDigit = 0xAB, kOpNonDigit = 0xAC, kOpMatch = 0xAD, kOpNotLiteral = 0xAE,
  kOpMaskedNotLiteral = 0xAF, kOpMatchAtEnd = 0xB0, kOpMatchAtStart = 0xB1,
  kOpWordBoundary = 0xB2, kOpNonWordBoundary = 0xB3, kOpRepeatAnyGreedy = 0xB4,
  kOpRepeatAnyUngreedy = 0xB5, kOpSplitA = 0xC0, kOpSplitB = 0xC1, kOpJump = 0xC2,
  kOpRepeatStartGreedy = 0xC3, kOpRepeatEndGreedy = 0xC4, kOpRepeatStartUngreedy = 0xC5,
  kOpRepeatEndUngreedy = 0xC6,
};

// Instruction size in bytes, 0 for an unknown opcode.
__host__ __device__ inline uint32_t re_op_size(uint8_t op) {
  switch (op) {
    case kOpAny: case kOpWordChar: case kOpNonWordChar: case kOpSpace: case kOpNonSpace:
    case kOpDigit: case kOpNonDigit: case kOpMatch: case kOpMatchAtEnd: case kOpMatchAtStart:
    case kOpWordBoundary: case kOpNonWordBoundary:
      return 1;
    case kOpLiteral: case kOpNotLiteral: return 2;
    case kOpMaskedLiteral: case kOpMaskedNotLiteral: return 3;
    case kOpClass: return 1 + 33;
    case kOpRepeatAnyGreedy: case kOpRepeatAnyUngreedy: return 1 + 4;
    case kOpSplitA: case kOpSplitB: return 1 + 1 + 2;
    case kOpJump: return 1 + 2;
    case kOpRepeatStartGreedy: case kOpRepeatEndGreedy: case kOpRepeatStartUngreedy:
    case kOpRepeatEndUngreedy:
      return 1 + 8;
    default: return 0;
  }
}

__host__ __device__ inline uint16_t re_u16(const uint8_t* p) { return (uint16_t)(p[0] | (p[1] << 8)); }
__host__ __device__ inline int16_t re_i16(const uint8_t* p) { return (int16_t)re_u16(p); }
__host__ __device__ inline int32_t re_i32(const uint8_t* p) {
  return (int32_t)((uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24));
}

// Host: extent of a yr_re_exec program (every reachable instruction inside
// [0, avail) and known), 0 if malformed.  scanner.cpp.
uint32_t re_general_extent(const uint8_t* code, uint64_t avail);

}  // namespace yamd
