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

/* Parameter presets (cpp/src/parameter_set.cpp:108-306, src/parameters/index.ts). */
const Q = {
  Q_60_1: 1152921504606584833n, Q_60_2: 1152921504598720513n, Q_60_3: 1152921504597016577n,
  Q_50_1: 1125899906826241n, Q_50_2: 1125899906793473n, Q_40_1: 1099511627777n, Q_40_2: 1099511562241n,
};
const PRESETS = {
  'tfhe-128-fast': { polyDegree: 1024, moduli: [Q.Q_40_1], lweDimension: 742, decompBaseLog: 23, decompLevel: 1 },
  'tfhe-128-balanced': { polyDegree: 2048, moduli: [Q.Q_50_1], lweDimension: 830, decompBaseLog: 15, decompLevel: 2 },
  'tfhe-256-secure': { polyDegree: 4096, moduli: [Q.Q_60_1], lweDimension: 1024, decompBaseLog: 10, decompLevel: 3 },
  'bfv-128-simd': { polyDegree: 8192, moduli: [Q.Q_60_1, Q.Q_60_2, Q.Q_60_3], decompBaseLog: 60, decompLevel: 3 },
  'ckks-128-ml': { polyDegree: 16384, moduli: [Q.Q_60_1, Q.Q_50_1, Q.Q_50_2, Q.Q_40_1, Q.Q_40_2],
    decompBaseLog: 40, decompLevel: 5 },
  'tfhe-128-voting': { polyDegree: 1024, moduli: [Q.Q_40_1], lweDimension: 742, decompBaseLog: 23, decompLevel: 1 },
};

/**
 * The ciphertext-arithmetic part of the TS FHEEngine (src/api/fhe-engine.ts:33-78)
 * on the GPU.  A ciphertext is a BigUint64Array [c0 | c1] (2n words), a
 * degree-2 product [c0 | c1 | c2] (3n words); batches concatenate them.
 * Every method returns a Promise like the reference interface.  Key
 * generation, encryption and serialisation are the reference's control
 * plane and stay in TS (out of scope for this backend).
 */
class GpuFHEEngine {
  constructor(params, { mode = 'compat', device = 0 } = {}) {
    this.params = params;
    this.ring = new PolynomialEngine(params.polyDegree, params.moduli[0], { mode, device });
    this.n = params.polyDegree;
  }
  async add(ct1, ct2) { return this.ring.add(ct1, ct2); }
  async subtract(ct1, ct2) { return this.ring.subtract(ct1, ct2); }
  async negate(ct) { return this.ring.negate(ct); }
  async multiplyScalar(ct, scalar) { return this.ring.multiplyScalar(ct, scalar); }
  async multiply(ct1, ct2) { return this.ring.ctMultiply(ct1, ct2); }
  async square(ct) { return this.ring.ctMultiply(ct, ct); }
  /** ct: degree-2 ciphertexts [batch][3][n]; ek: BigUint64Array [level][2][n]
   *  (a_l, b_l) key-switch pairs.  { degree: 1 } returns a copy, as the
   *  reference does for a degree-1 input (encryption.cpp:906-909). */
  async relinearize(ct, ek, baseLog = this.params.decompBaseLog || 4, { degree = 2 } = {}) {
    if (degree === 1) return BigUint64Array.from(ct);
    return this.ring.relinearize(ct, ek, baseLog);
  }
  async multiplyRelin(ct1, ct2, ek, baseLog) { return this.relinearize(await this.multiply(ct1, ct2), ek, baseLog); }
  async squareRelin(ct, ek, baseLog) { return this.relinearize(await this.square(ct), ek, baseLog); }
  /** pt: encoded plaintext polynomial (n words), applied to both components */
  async multiplyPlain(ct, pt) {
    const rep = new BigUint64Array(ct.length);
    for (let off = 0; off < ct.length; off += this.n) rep.set(pt, off);
    return this.ring.multiply(ct, rep);
  }
  getParams() { return this.params; }
  getHardwareCapabilities() { return native.detectHardware(); }
  dispose() { this.ring = null; }
}

/** createEngine (src/index.ts:108): a preset name or custom parameters. */
async function createEngine(params, options) {
  const p = typeof params === 'string' ? PRESETS[params] : params;
  if (!p) throw new RangeError(`Unknown parameter preset: ${params}`);
  return new GpuFHEEngine(p, options);
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
  GpuFHEEngine,
  createEngine,
  PRESETS,
};
