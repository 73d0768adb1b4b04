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
const { envDefaults } = require('./engine');

/**
 * Batched polynomial arithmetic over Z_q[X] for the TS FHEEngine
 * (src/api/fhe-engine.ts:33-78): contiguous BigUint64Array buffers of
 * batch * degree coefficients (the reference Polynomial layout).
 */
class PolynomialEngine {
  constructor(degree, modulus, opts = {}) {
    const { mode, device } = envDefaults(opts);
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
  /** ciphertexts of two-CU blind rotations recomputed by the one-CU repair pass */
  brRepairCount() { return this.ctx.brRepairCount(); }
  info() { return this.ctx.info(); }
}

/* Parameter presets (cpp/src/parameter_set.cpp:108-306, src/parameters/index.ts). */
const Q = {
  Q_60_1: 1152921504606584833n, Q_60_2: 1152921504598720513n, Q_60_3: 1152921504597016577n,
  Q_50_1: 1125899906826241n, Q_50_2: 1125899906793473n, Q_40_1: 1099511627777n, Q_40_2: 1099511562241n,
};
const PRESETS = {
  'tfhe-128-fast': { polyDegree: 1024, moduli: [Q.Q_40_1], plaintextModulus: 4, lweDimension: 742, decompBaseLog: 23, decompLevel: 1 },
  'tfhe-128-balanced': { polyDegree: 2048, moduli: [Q.Q_50_1], plaintextModulus: 8, lweDimension: 830, decompBaseLog: 15, decompLevel: 2 },
  'tfhe-256-secure': { polyDegree: 4096, moduli: [Q.Q_60_1], plaintextModulus: 16, lweDimension: 1024, decompBaseLog: 10, decompLevel: 3 },
  'bfv-128-simd': { polyDegree: 8192, moduli: [Q.Q_60_1, Q.Q_60_2, Q.Q_60_3], plaintextModulus: 65537,
    decompBaseLog: 60, decompLevel: 3 },
  'ckks-128-ml': { polyDegree: 16384, moduli: [Q.Q_60_1, Q.Q_50_1, Q.Q_50_2, Q.Q_40_1, Q.Q_40_2],
    plaintextModulus: 2n ** 40n,
    decompBaseLog: 40, decompLevel: 5 },
  'tfhe-128-voting': { polyDegree: 1024, moduli: [Q.Q_40_1], plaintextModulus: 16, lweDimension: 742, decompBaseLog: 23, decompLevel: 1 },
};

/* ---- host-side sampling (SecureRandom, key_manager.cpp:38-120): the
 * control plane samples, the GPU computes.  Not bit-exact with the
 * reference's random device (nothing random is); callers that need
 * determinism pass their own u / e1 / e2 to encrypt(). */
const crypto = require('crypto');
function randomU64s(count) {
  const out = new BigUint64Array(count);
  crypto.randomFillSync(out);
  return out;
}
/* random_u64_range (:60-71): rejection sampling, then % max */
function uniformMod(q, count) {
  const out = randomU64s(count);
  const thr = ((1n << 64n) - q) % q;
  for (let i = 0; i < count; i++) {
    while (out[i] < thr) out[i] = randomU64s(1)[0];
    out[i] %= q;
  }
  return out;
}
/* sample_ternary (:73-83): {q-1, 0, 1} */
function ternary(q, count) {
  const r = uniformMod(3n, count);
  for (let i = 0; i < count; i++) r[i] = r[i] === 0n ? q - 1n : r[i] === 1n ? 0n : 1n;
  return r;
}
/* sample_gaussian (:85-110): Box-Muller, rounded, negatives as q + x */
function gaussian(q, std, count) {
  const out = new BigUint64Array(count);
  const u = randomU64s(2 * count);
  for (let i = 0; i < count; i++) {
    let u1 = Number(u[2 * i] >> 11n) / 2 ** 53;
    const u2 = Number(u[2 * i + 1] >> 11n) / 2 ** 53;
    if (u1 === 0) u1 = 2 ** -53;
    const z = Math.round(Math.sqrt(-2 * Math.log(u1)) * Math.cos(2 * Math.PI * u2) * std);
    out[i] = z < 0 ? q + BigInt(z) : BigInt(z);
  }
  return out;
}

/**
 * The TS FHEEngine (src/index.ts:84-105, src/api/fhe-engine.ts:33-78) on the
 * GPU.  A ciphertext is a BigUint64Array [c0 | c1] (2n words), a degree-2
 * product [c0 | c1 | c2] (3n words); batches concatenate them.  Every
 * method returns a Promise and runs as napi_async_work (the `...Async`
 * native forms): the event loop is never blocked by a transfer or kernel.
 * Keys: { poly, prep } objects from generateSecretKey / generatePublicKey
 * (prep = the NTT-domain form the kernels consume) and { rlk, baseLog,
 * level } from generateEvalKey.  Serialisation and key management stay in
 * the reference's TS control plane (out of scope for this backend).
 */
class GpuFHEEngine {
  constructor(params, opts = {}) {
    const { mode, device, devices } = envDefaults(opts);
    this.params = params;
    this.n = params.polyDegree;
    this.q = BigInt(params.moduli[0]);
    this.t = BigInt(params.plaintextModulus || 0);
    this.noiseStd = params.lweNoiseStd || 3.2;
    const m = mode === 'negacyclic' ? 1 : mode === 'compat' ? 0 : -1;
    if (m < 0) throw new RangeError(`unknown mode ${mode}`);
    this.ctx = new native.NttContext(this.n, this.q, m, devices || device);
    this.ring = new PolynomialEngine(this.n, this.q, { mode, device });
    this.ring.ctx = this.ctx;
  }
  _alloc(words) { return new BigUint64Array(words); }
  _batch(ct, comps = 2) { return ct.length / (comps * this.n); }

  // ---- keys (key_manager.cpp:150-330)
  async generateSecretKey() {
    const poly = ternary(this.q, this.n);
    return this.importSecretKey(poly);
  }
  async importSecretKey(poly) {
    const prep = await this.ctx.prepareSecretKeyAsync(poly, this._alloc(2 * this.n));
    return { poly, prep };
  }
  /** pk = (a, b = a s + e) */
  async generatePublicKey(sk, { a = uniformMod(this.q, this.n), e = gaussian(this.q, this.noiseStd, this.n) } = {}) {
    const as = await this.ctx.polymulAsync(a, sk.poly, this._alloc(this.n));
    const b = await this.ctx.addAsync(as, e, this._alloc(this.n));
    return this.importPublicKey(a, b);
  }
  async importPublicKey(a, b) {
    const poly = this._alloc(2 * this.n);
    poly.set(a, 0);
    poly.set(b, this.n);
    const prep = await this.ctx.preparePublicKeyAsync(poly, this._alloc(2 * this.n));
    return { a, b, poly, prep };
  }
  /** generate_eval_key (:233-330): (a_l, b_l = a_l s + e_l + s^2 base^l);
   *  levels limited to (level - 1) * baseLog < 64 (a digit shift of 64 or
   *  more is undefined in the reference's relinearize). */
  async generateEvalKey(sk, decompBaseLog = this.params.decompBaseLog || 4, { level, a: aIn, e: eIn } = {}) {
    const bl = decompBaseLog;
    const lv = Math.min(level || this.params.decompLevel || 3, Math.floor(63 / bl) + 1);
    const n = this.n;
    const s2 = await this.ctx.polymulAsync(sk.poly, sk.poly, this._alloc(n));
    const rlk = this._alloc(lv * 2 * n);
    let power = 1n;
    for (let l = 0; l < lv; l++) {
      const a = aIn ? aIn[l] : uniformMod(this.q, n);  // caller-supplied samples: deterministic keys
      const e = eIn ? eIn[l] : gaussian(this.q, this.noiseStd, n);
      const as = await this.ctx.polymulAsync(a, sk.poly, this._alloc(n));
      const b = await this.ctx.addAsync(as, e, this._alloc(n));
      const sc = await this.ctx.mulScalarAsync(s2, power, this._alloc(n));
      rlk.set(a, 2 * l * n);
      rlk.set(await this.ctx.addAsync(b, sc, this._alloc(n)), (2 * l + 1) * n);
      power = (power * (1n << BigInt(bl))) % this.q;
    }
    return { rlk, baseLog: bl, level: lv };
  }

  // ---- plaintexts (encode_plaintext / encode_packed take raw slot values)
  getSlotCount() { return this.n; }
  createPlaintext(value) { const p = this._alloc(this.n); p[0] = BigInt(value); return p; }
  createPackedPlaintext(values) {
    const p = this._alloc(this.n);
    values.slice(0, this.n).forEach((v, i) => { p[i] = BigInt(v); });
    return p;
  }

  // ---- encrypt / decrypt (encryption.cpp:171-348)
  /** pt: slot values (n words per ciphertext, batches concatenate) or a bigint */
  async encrypt(pt, pk, { u, e1, e2 } = {}) {
    const slots = typeof pt === 'bigint' || typeof pt === 'number' ? this.createPlaintext(pt) : pt;
    const words = slots.length;
    u = u || ternary(this.q, words);
    e1 = e1 || gaussian(this.q, this.noiseStd, words);
    e2 = e2 || gaussian(this.q, this.noiseStd, words);
    return this.ctx.encryptAsync(this.t, pk.prep, slots, u, e1, e2, this._alloc(2 * words));
  }
  async encryptValue(value, pk) { return this.encrypt(this.createPlaintext(value), pk); }
  async encryptPacked(values, pk) { return this.encrypt(this.createPackedPlaintext(values), pk); }
  async batchEncrypt(pts, pk) {
    const all = this._alloc(pts.length * this.n);
    pts.forEach((p, i) => all.set(typeof p === 'bigint' ? this.createPlaintext(p) : p, i * this.n));
    return this.encrypt(all, pk);
  }
  /** -> { values (slots, per ciphertext), maxNoise, noiseBudget[], success[] } */
  async decrypt(ct, sk, { degree = 1, isNtt = false, phase = false } = {}) {
    const comps = degree === 2 ? 3 : 2;
    const batch = this._batch(ct, comps);
    const values = this._alloc(batch * this.n), maxNoise = this._alloc(batch);
    const ph = phase ? this._alloc(batch * this.n) : undefined;
    await this.ctx.decryptAsync(this.t, sk.prep, ct, comps, isNtt ? 1 : 0, values, maxNoise, ph);
    const qd = Number(this.q);
    const noiseBudget = Array.from(maxNoise, (m) => Math.log2(qd / (2 * Math.max(Number(m), 1))));
    return { values, maxNoise, noiseBudget, success: noiseBudget.map((b) => b >= 0), phase: ph };
  }
  async decryptValue(ct, sk, opts) {
    const r = await this.decrypt(ct, sk, opts);
    if (!r.success[0]) throw new Error('Noise budget exhausted - decryption may be incorrect');
    return r.values[0];
  }
  async decryptPacked(ct, sk, numValues, opts) {
    const r = await this.decrypt(ct, sk, opts);
    return Array.from(r.values.slice(0, numValues));
  }
  async getNoiseBudget(ct, sk, opts) { return (await this.decrypt(ct, sk, opts)).noiseBudget[0]; }

  // ---- homomorphic arithmetic (encryption.cpp:594-980)
  async add(ct1, ct2) { return this.ctx.addAsync(ct1, ct2, this._alloc(ct1.length)); }
  async subtract(ct1, ct2) { return this.ctx.subAsync(ct1, ct2, this._alloc(ct1.length)); }
  async negate(ct) { return this.ctx.negateAsync(ct, this._alloc(ct.length)); }
  async multiplyScalar(ct, scalar) { return this.ctx.mulScalarAsync(ct, BigInt(scalar), this._alloc(ct.length)); }
  async addPlain(ct, pt, { isNtt = false } = {}) {
    const slots = typeof pt === 'bigint' || typeof pt === 'number' ? this.createPlaintext(pt) : pt;
    const batch = this._batch(ct);
    let vals = slots;
    if (slots.length !== batch * this.n) {  // one plaintext for every ciphertext
      vals = this._alloc(batch * this.n);
      for (let i = 0; i < batch; i++) vals.set(slots, i * this.n);
    }
    return this.ctx.addPlainAsync(this.t, ct, vals, isNtt ? 1 : 0, this._alloc(ct.length));
  }
  async multiply(ct1, ct2, { isNtt = false } = {}) {
    return this.ctx.ctMultiplyAsync(ct1, ct2, this._alloc(ct1.length / 2 * 3), isNtt ? 1 : 0);
  }
  async square(ct) { return this.multiply(ct, ct); }
  /** ct: degree-2 ciphertexts [batch][3][n]; ek: generateEvalKey's key or a
   *  BigUint64Array [level][2][n] of (a_l, b_l).  { degree: 1 } returns a
   *  copy, as the reference does for a degree-1 input (encryption.cpp:906-909). */
  async relinearize(ct, ek, baseLog, { degree = 2 } = {}) {
    if (degree === 1) return BigUint64Array.from(ct);
    const rlk = ek.rlk || ek;
    const bl = baseLog || ek.baseLog || this.params.decompBaseLog || 4;
    return this.ctx.relinearizeAsync(ct, rlk, bl, this._alloc(ct.length / 3 * 2));
  }
  async multiplyRelin(ct1, ct2, ek, baseLog) { return this.relinearize(await this.multiply(ct1, ct2), ek, baseLog); }
  async squareRelin(ct, ek, baseLog) { return this.relinearize(await this.square(ct), ek, baseLog); }
  /** pt: encoded plaintext polynomial (n words), applied to both components */
  async multiplyPlain(ct, pt) {
    const rep = this._alloc(ct.length);
    for (let off = 0; off < ct.length; off += this.n) rep.set(pt, off);
    return this.ctx.polymulAsync(ct, rep, this._alloc(ct.length));
  }

  // ---- TFHE bootstrap (bootstrap_engine.cpp:684-722), k = 1
  /** lwe: { a: BigUint64Array [batch*dim], b: BigUint64Array [batch] };
   *  bk: { bsk [dim][2*level][2][n] (coefficient-form GGSWs), baseLog, level,
   *        kskA [n*ksLevel][outDim], kskB [n*ksLevel], ksBaseLog, ksLevel,
   *        testPoly? (n words; default: the identity lookup table) } */
  async bootstrap(lwe, bk, testPoly) {
    const n = this.n, batch = lwe.b.length;
    const tp = testPoly || bk.testPoly || this.createLookupTable((x) => x, 4, 4);
    const outDim = bk.kskA.length / (n * bk.ksLevel);
    const a = this._alloc(batch * outDim), b = this._alloc(batch);
    await this.ctx.bootstrapAsync(lwe.a, lwe.b, bk.bsk, tp, bk.kskA, bk.kskB, bk.baseLog, bk.level, bk.ksBaseLog,
      bk.ksLevel, a, b);
    return { a, b };
  }
  async programmableBootstrap(lwe, bk, lut) { return this.bootstrap(lwe, bk, lut); }
  /** create_lookup_table (bootstrap_engine.cpp:725-758) */
  createLookupTable(fn, inputModulus, outputModulus) {
    const n = this.n, q = this.q, deltaOut = q / BigInt(outputModulus);
    const c = this._alloc(n);
    for (let i = 0; i < n; i++) {
      const v = BigInt(Math.floor((i * inputModulus + n) / (2 * n)) % inputModulus);
      c[i] = ((BigInt(fn(v)) % BigInt(outputModulus)) * deltaOut) % q;
    }
    return c;
  }

  getParams() { return this.params; }
  getHardwareCapabilities() { return native.detectHardware(); }
  dispose() { this.ring = null; this.ctx = null; }
}

/* createEngine (src/index.ts:108, api/fhe-engine.ts:464-476): a preset name
 * or custom parameters -> the FHEEngine surface with device-resident
 * handles (lib/engine.js).  GpuFHEEngine above is the array-level engine
 * (raw BigUint64Array ciphertexts, caller-supplied randomness) kept for
 * batch callers and the golden tests. */
const engine = require('./engine');
const { createEngine, FHEEngineImpl } = engine.makeEngineClass(native);

module.exports = {
  initialize: native.initialize,
  detectHardware: native.detectHardware,
  version: native.version,
  ModularArithmetic: native.ModularArithmetic,
  NttContext: native.NttContext,
  DeviceBuffer: native.DeviceBuffer,
  modmulBatch: native.modmulBatch,
  mlMontgomeryMulBatch: native.mlMontgomeryMulBatch,
  PolynomialEngine,
  GpuFHEEngine,
  FHEEngineImpl,
  createEngine,
  createFHEEngine: createEngine,
  createParameterSet: engine.createParameterSet,
  getAvailablePresets: engine.getAvailablePresets,
  calculateDerivedParameters: engine.calculateDerivedParameters,
  NTT_PRIMES: engine.NTT_PRIMES,
  FHEError: engine.FHEError,
  FHEErrorCode: engine.FHEErrorCode,
  PRESETS,
  sampling: { uniformMod, ternary, gaussian },
};
