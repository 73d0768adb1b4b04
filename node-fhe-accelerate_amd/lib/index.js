'use strict';
/**
 * node-fhe-accelerate (MI355X backend) -- JS entry point.
 *
 * Same exports as the reference's napi-rs module (index.d.ts:14-44):
 *   initialize(), detectHardware(), version(), ModularArithmetic
 * plus the batched polynomial engine backed by libfhe_gpu.so:
 *   NttContext, modmulBatch, mlMontgomeryMulBatch, PolynomialEngine.
 */
const path = require('path');

const native = require(process.env.FHE_NAPI_PATH || path.join(__dirname, '..', 'build', 'fhe_napi.node'));

/**
 * Batched polynomial arithmetic over Z_q[X] for the TS FHEEngine
 * (src/api/fhe-engine.ts:33-78): contiguous BigUint64Array buffers of
 * batch * degree coefficients (the reference Polynomial layout).
 */
class PolynomialEngine {
  constructor(degree, modulus, { mode = 'compat', device = 0 } = {}) {
    const m = mode === 'negacyclic' ? 1 : mode === 'compat' ? 0 : -1;
    if (m < 0) throw new RangeError(`unknown mode ${mode}`);
    this.ctx = new native.NttContext(degree, BigInt(modulus), m, device);
    this.degree = degree;
    this.modulus = BigInt(modulus);
  }
  alloc(batch = 1) { return new BigUint64Array(batch * this.degree); }
  toNtt(a, out) { return this.ctx.forward(a, out); }
  fromNtt(a, out) { return this.ctx.inverse(a, out); }
  multiply(a, b, out = this.alloc(a.length / this.degree)) { return this.ctx.polymul(a, b, out); }
  pointwiseMultiply(a, b, out = this.alloc(a.length / this.degree)) { return this.ctx.pointwise(a, b, out); }
  add(a, b, out = this.alloc(a.length / this.degree)) { return this.ctx.add(a, b, out); }
  subtract(a, b, out = this.alloc(a.length / this.degree)) { return this.ctx.sub(a, b, out); }
  negate(a, out = this.alloc(a.length / this.degree)) { return this.ctx.negate(a, out); }
  multiplyScalar(a, s, out = this.alloc(a.length / this.degree)) { return this.ctx.mulScalar(a, BigInt(s), out); }
  forwardMultiply(a, w, out = this.alloc(a.length / this.degree)) { return this.ctx.forwardMul(a, w, out); }
  externalProduct(glwe, ggsw, baseLog, level, out = new BigUint64Array(glwe.length)) {
    return this.ctx.externalProduct(glwe, ggsw, baseLog, level, out);
  }
  /** EncryptionEngine::multiply: ct [batch][2][n] -> [batch][3][n] */
  ctMultiply(ct1, ct2, { isNtt = false } = {}, out = new BigUint64Array(ct1.length / 2 * 3)) {
    return this.ctx.ctMultiply(ct1, ct2, out, isNtt ? 1 : 0);
  }
  /** EncryptionEngine::relinearize: ct3 [batch][3][n], rlk [level][2][n] (a_l, b_l) */
  relinearize(ct3, rlk, baseLog = 4, out = new BigUint64Array(ct3.length / 3 * 2)) {
    return this.ctx.relinearize(ct3, rlk, baseLog, out);
  }
  /** EncryptionEngine::multiply_relin */
  multiplyRelin(ct1, ct2, rlk, baseLog = 4) {
    return this.relinearize(this.ctMultiply(ct1, ct2), rlk, baseLog);
  }
  /** BootstrapEngine::blind_rotate (k = 1), in place on acc [batch][2][n] */
  blindRotate(acc, lweA, lweB, bsk, baseLog, level) {
    return this.ctx.blindRotate(acc, lweA, lweB, bsk, baseLog, level);
  }
  info() { return this.ctx.info(); }
}

module.exports = {
  initialize: native.initialize,
  detectHardware: native.detectHardware,
  version: native.version,
  ModularArithmetic: native.ModularArithmetic,
  NttContext: native.NttContext,
  modmulBatch: native.modmulBatch,
  mlMontgomeryMulBatch: native.mlMontgomeryMulBatch,
  PolynomialEngine,
};
