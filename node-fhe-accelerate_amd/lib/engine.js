'use strict';
/**
 * The TypeScript FHEEngine surface (src/api/fhe-engine.ts:33-78,
 * src/api/types.ts:18-166) on the MI355X backend.
 *
 * Every key and ciphertext is a branded, frozen handle object of the
 * reference's shape -- Ciphertext {__brand, handle, keyId, noiseBudget, isNtt,
 * degree}, SecretKey / PublicKey {__brand, handle, keyId}, EvaluationKey
 * {..., decompBaseLog, decompLevel}, BootstrapKey {..., lweDimension} --
 * whose `handle` is the HBM address of its native DeviceBuffer.  The words
 * stay on the GPU between operations: encrypt draws u / e1 / e2 on the
 * device (seeded ChaCha20, fhe_encrypt_sampled_batch), every homomorphic
 * operation is a device-to-device kernel call, and only decrypt /
 * serialisation bring words back.  Device memory is released when the
 * handle object is collected (N-API finalizer, stream-ordered free).
 *
 * Semantics follow the reference C++ engines the TS surface fronts:
 * EncryptionEngine (encryption.cpp: encode/decode, encrypt_internal,
 * decrypt + compute_noise_budget, add/subtract/negate/add_plain/add_scalar,
 * multiply/multiply_plain/multiply_scalar/relinearize and their noise-budget
 * bookkeeping), KeyManager (key_manager.cpp: generate_secret_key /
 * public / eval / threshold keys, partial decryption, Lagrange combination)
 * and BootstrapEngine (bootstrap_engine.cpp: generate_bootstrap_key,
 * bootstrap_with_test_poly, create_lookup_table, the identity test
 * polynomial).  Parameter sets are parameters/index.ts's presets.
 *
 * Randomness: SecureRandom's draws come from a ChaCha20 stream keyed by a
 * 256-bit seed (crypto.randomBytes unless createEngine's options.seed fixes
 * it: then every key and ciphertext is reproducible, which the parity tests
 * use), each key / encryption taking fresh stream ids.
 */
const crypto = require('crypto');
const zlib = require('zlib');

const M64 = (1n << 64n) - 1n;

// ---------------------------------------------------------------- errors (types.ts:140-166)
const FHEErrorCode = Object.freeze({
  NOISE_BUDGET_EXHAUSTED: 'NOISE_BUDGET_EXHAUSTED',
  INVALID_PARAMETERS: 'INVALID_PARAMETERS',
  KEY_MISMATCH: 'KEY_MISMATCH',
  HARDWARE_UNAVAILABLE: 'HARDWARE_UNAVAILABLE',
  SERIALIZATION_ERROR: 'SERIALIZATION_ERROR',
  PROOF_VERIFICATION_FAILED: 'PROOF_VERIFICATION_FAILED',
  THRESHOLD_NOT_MET: 'THRESHOLD_NOT_MET',
  INVALID_BALLOT: 'INVALID_BALLOT',
  DUPLICATE_VOTE: 'DUPLICATE_VOTE',
  NATIVE_ERROR: 'NATIVE_ERROR',
});

class FHEError extends Error {
  constructor(message, code, details) {
    super(message);
    this.name = 'FHEError';
    this.code = code;
    this.details = details;
    Object.setPrototypeOf(this, FHEError.prototype);
  }
}

/** Native errors carry a FHEErrorCode name in `code` (fhe_napi.c code_name). */
function toFHEError(e) {
  if (e instanceof FHEError) return e;
  const code = e && FHEErrorCode[e.code] ? e.code : FHEErrorCode.NATIVE_ERROR;
  return new FHEError(e && e.message ? e.message : String(e), code,
    e && e.status !== undefined ? { status: e.status } : undefined);
}
async function guard(fn) {
  try {
    return await fn();
  } catch (e) {
    throw toFHEError(e);
  }
}

// ---------------------------------------------------------------- parameter sets (parameters/index.ts)
const NTT_PRIMES = Object.freeze({
  Q_60_1: 1152921504606584833n, Q_60_2: 1152921504598720513n, Q_60_3: 1152921504597016577n,
  Q_50_1: 1125899906826241n, Q_50_2: 1125899906793473n,
  Q_40_1: 1099511627777n, Q_40_2: 1099511562241n,
  Q_30_1: 1073479681n, Q_30_2: 1073217537n,
});

/** calculateDerivedParameters (parameters/index.ts:91-124) */
function calculateDerivedParameters(p) {
  let logQ = 0;
  for (const q of p.moduli || []) logQ += Math.log2(Number(q));
  const logT = Math.log2(Number(p.plaintextModulus || 1n));
  let noiseBudget;
  if (p.scheme === 'TFHE') {
    noiseBudget = logQ - Math.log2((p.lweNoiseStd || 1) * Math.sqrt(p.lweDimension || 1)) - 10;
  } else {
    noiseBudget = logQ - logT - 20;
  }
  noiseBudget = Math.max(0, noiseBudget);
  let maxMultDepth = Math.floor(noiseBudget / 10);
  if (p.scheme === 'TFHE' && (p.decompLevel || 0) > 0) maxMultDepth = 1000;
  return { noiseBudget, maxMultDepth };
}
function preset(scheme, security, polyDegree, moduli, lweDimension, lweNoiseStd, decompBaseLog, decompLevel,
  plaintextModulus) {
  const p = {
    scheme, security, polyDegree, moduli, lweDimension, lweNoiseStd, glweDimension: 1, decompBaseLog,
    decompLevel, plaintextModulus, noiseBudget: 0, maxMultDepth: 0,
  };
  Object.assign(p, calculateDerivedParameters(p));
  return p;
}
const Q = NTT_PRIMES;
const PRESET_FACTORIES = {
  'tfhe-128-fast': () => preset('TFHE', 128, 1024, [Q.Q_40_1], 742, 3.2e-11, 23, 1, 4n),
  'tfhe-128-balanced': () => preset('TFHE', 128, 2048, [Q.Q_50_1], 830, 2.9e-11, 15, 2, 8n),
  'tfhe-256-secure': () => preset('TFHE', 256, 4096, [Q.Q_60_1], 1024, 2.0e-12, 10, 3, 16n),
  'bfv-128-simd': () => preset('BFV', 128, 8192, [Q.Q_60_1, Q.Q_60_2, Q.Q_60_3], 0, 3.2, 60, 3, 65537n),
  'ckks-128-ml': () => preset('CKKS', 128, 16384, [Q.Q_60_1, Q.Q_50_1, Q.Q_50_2, Q.Q_40_1, Q.Q_40_2], 0, 3.2, 40, 5,
    1n << 40n),
  'tfhe-128-voting': () => preset('TFHE', 128, 1024, [Q.Q_40_1], 742, 3.2e-11, 23, 1, 16n),
};
/** createParameterSet / createCustomParameterSet (parameters/index.ts:296-347) */
function createParameterSet(params) {
  if (typeof params === 'string') {
    const f = PRESET_FACTORIES[params];
    if (!f) throw new FHEError(`Unknown parameter preset: ${params}`, FHEErrorCode.INVALID_PARAMETERS);
    return f();
  }
  if (!params || typeof params !== 'object' || !params.polyDegree || !params.moduli || !params.moduli.length) {
    throw new FHEError('Custom parameters need polyDegree and moduli', FHEErrorCode.INVALID_PARAMETERS);
  }
  const p = {
    scheme: params.scheme || (params.lweDimension ? 'TFHE' : 'BFV'),
    security: params.securityLevel || params.security || 128,
    polyDegree: params.polyDegree,
    moduli: params.moduli.map((m) => BigInt(m)),
    lweDimension: params.lweDimension || 0,
    lweNoiseStd: params.lweNoiseStd || 3.2e-11,
    glweDimension: params.glweDimension || 1,
    decompBaseLog: params.decompBaseLog || 23,
    decompLevel: params.decompLevel || 1,
    // createCustomParameterSet fixes t = 4; an explicit plaintextModulus is kept
    plaintextModulus: params.plaintextModulus !== undefined ? BigInt(params.plaintextModulus) : 4n,
    noiseBudget: 0,
    maxMultDepth: 0,
  };
  Object.assign(p, calculateDerivedParameters(p));
  return p;
}
function getAvailablePresets() {
  return ['tfhe-128-fast', 'tfhe-128-balanced', 'tfhe-256-secure', 'bfv-128-simd', 'ckks-128-ml'];
}

// ---------------------------------------------------------------- helpers
const SAMPLE = { UNIFORM: 0, TERNARY: 1, GAUSSIAN: 2, BINARY: 3, RAW: 4 };
const DIST = { TERNARY: SAMPLE.TERNARY, GAUSSIAN: SAMPLE.GAUSSIAN, BINARY: SAMPLE.BINARY, UNIFORM: SAMPLE.UNIFORM };
const SERIAL_MAGIC = 0x4d454846; // 'FHEM'
const KINDS = ['ciphertext', 'secret', 'public', 'evaluation', 'bootstrap'];

function u64(v) { return BigInt.asUintN(64, BigInt(v)); }
function modPow(b, e, m) {
  let r = 1n;
  b %= m;
  while (e > 0n) {
    if (e & 1n) r = (r * b) % m;
    b = (b * b) % m;
    e >>= 1n;
  }
  return r;
}
function toBigIntArray(words, count) {
  const out = new Array(count);
  for (let i = 0; i < count; i++) out[i] = words[i];
  return out;
}

/**
 * createEngine(params, options?) -> Promise<FHEEngine>
 * options: { mode: 'compat' | 'negacyclic', device, seed (Uint8Array(32) | bigint) }
 */
function makeEngineClass(native) {
  const { NttContext, DeviceBuffer } = native;
  // native state of every handle object (spread copies are not handles)
  const state = new WeakMap();

  class FHEEngineImpl {
    constructor(params, options) {
      const o = options || {};
      this._params = params;
      this._n = params.polyDegree;
      this._q = BigInt(params.moduli[0]);
      this._t = params.plaintextModulus ? BigInt(params.plaintextModulus) : 4n;
      this._tEff = this._t === 0n ? 4n : this._t;
      this._delta = this._q / this._tEff;
      // the C++ engines' error std (encryption.cpp:52-56: lwe_noise_std or 3.2)
      this._std = params.lweNoiseStd > 0 ? params.lweNoiseStd : 3.2;
      this._initialBudget = Math.log2(Number(this._q)) - Math.log2(2 * this._std * Math.sqrt(this._n));
      let env;
      try {
        env = envDefaults(o);
      } catch (err) {
        throw new FHEError(err.message, FHEErrorCode.INVALID_PARAMETERS);
      }
      const mode = env.mode === 'negacyclic' ? 1 : env.mode === 'compat' ? 0 : -1;
      if (mode < 0) throw new FHEError(`unknown mode ${env.mode}`, FHEErrorCode.INVALID_PARAMETERS);
      this._mode = mode;
      this._ctx = new NttContext(this._n, this._q, mode, env.devices || env.device);
      let seed = o.seed;
      if (seed === undefined) seed = crypto.randomBytes(32);
      if (typeof seed === 'bigint' || typeof seed === 'number') {
        const s = new BigUint64Array(4);
        let v = BigInt(seed);
        for (let i = 0; i < 4; i++) { s[i] = v & M64; v >>= 64n; }
        this._seed = s;
      } else {
        const b = Buffer.alloc(32);
        Buffer.from(seed).copy(b);
        this._seed = new BigUint64Array(b.buffer.slice(b.byteOffset, b.byteOffset + 32));
      }
      this._stream = 1n;
      this._nextKey = BigInt(Date.now()) * 1000n;
      this._disposed = false;
    }

    // ---- plumbing
    _check() {
      if (this._disposed) throw new FHEError('Engine disposed', FHEErrorCode.NATIVE_ERROR);
    }
    _streams(k) { const s = this._stream; this._stream += BigInt(k); return s; }
    _keyId() { this._nextKey += 1n; return this._nextKey; }
    _buf(words) { return new DeviceBuffer(this._ctx, words); }
    _upload(words) { return this._buf(words.length).upload(words); }
    _st(h, brand) {
      const s = h && typeof h === 'object' ? state.get(h) : undefined;
      if (!s || h.__brand !== brand || s.engine !== this) {
        throw new FHEError(`not a ${brand} handle of this engine`, FHEErrorCode.INVALID_PARAMETERS);
      }
      return s;
    }
    _handle(brand, fields, st) {
      const h = Object.assign({ __brand: brand, handle: st.buf ? st.buf.handle : 0n }, fields);
      st.engine = this;
      Object.freeze(h);
      state.set(h, st);
      return h;
    }
    _ct(buf, keyId, noiseBudget, degree, extra) {
      return this._handle('Ciphertext', { keyId, noiseBudget, isNtt: false, degree },
        Object.assign({ buf, kind: 'rlwe', comps: degree + 1, packed: false }, extra || {}));
    }
    _sameKey(a, b, what) {
      if (a.keyId !== b.keyId) throw new FHEError(`Cannot ${what} ciphertexts encrypted with different keys`, FHEErrorCode.KEY_MISMATCH);
    }
    _rlwe(ct) {
      const s = this._st(ct, 'Ciphertext');
      if (s.kind !== 'rlwe') throw new FHEError('operation needs an RLWE ciphertext (not a bootstrapped LWE one)', FHEErrorCode.INVALID_PARAMETERS);
      return s;
    }
    /** encode_plaintext / encode_packed slots (encryption.cpp:107-131): the raw
     *  slot values, n per ciphertext; the kernels scale by delta */
    _slots(pt) {
      if (!pt || pt.__brand !== 'Plaintext' || !Array.isArray(pt.values)) {
        throw new FHEError('expected a Plaintext', FHEErrorCode.INVALID_PARAMETERS);
      }
      const s = new BigUint64Array(this._n);
      if (pt.isPacked && pt.values.length > 1) {
        const m = Math.min(pt.values.length, this._n);
        for (let i = 0; i < m; i++) s[i] = u64(pt.values[i]);
      } else {
        s[0] = u64(pt.values.length ? pt.values[0] : 0n);
      }
      return s;
    }
    /** the encoded polynomial (v * delta mod 2^64) mod q of encode_* */
    _encoded(pt) {
      const s = this._slots(pt);
      for (let i = 0; i < s.length; i++) if (s[i]) s[i] = ((s[i] * this._delta) & M64) % this._q;
      return s;
    }
    _budgetOf(maxNoise) {
      const m = Math.max(Number(maxNoise), 1);
      return Math.log2(Number(this._q) / (2 * m));
    }

    // ---- keys (key_manager.cpp)
    async generateSecretKey(options) {
      this._check();
      return guard(async () => {
        const dist = options && options.distribution ? DIST[options.distribution] : SAMPLE.TERNARY;
        if (dist === undefined) throw new FHEError(`unknown distribution ${options.distribution}`, FHEErrorCode.INVALID_PARAMETERS);
        const sk = this._buf(this._n);
        await this._ctx.sampleAsync(dist, this._seed, this._streams(1), this._std, sk);
        const prep = this._buf(2 * this._n);
        await this._ctx.prepareSecretKeyAsync(sk, prep);
        return this._handle('SecretKey', { keyId: this._keyId() }, { buf: sk, prep });
      });
    }
    async generatePublicKey(sk) {
      this._check();
      return guard(async () => {
        const s = this._st(sk, 'SecretKey');
        const pk = this._buf(2 * this._n);
        await this._ctx.publicKeyGenerateAsync(s.buf, this._seed, this._streams(2), this._std, pk);
        const prep = this._buf(2 * this._n);
        await this._ctx.preparePublicKeyAsync(pk, prep);
        return this._handle('PublicKey', { keyId: sk.keyId }, { buf: pk, prep });
      });
    }
    /** generate_eval_key (:252-333); levels limited to (level - 1) * baseLog < 64
     *  (relinearize's digit shift) */
    async generateEvalKey(sk, options) {
      this._check();
      return guard(async () => {
        const s = this._st(sk, 'SecretKey');
        const o = typeof options === 'number' ? { decompBaseLog: options } : (options || {});
        const bl = o.decompBaseLog || this._params.decompBaseLog || 4;
        const lv = Math.min(o.decompLevel || this._params.decompLevel || 3, Math.floor(63 / bl) + 1);
        if (bl < 1 || bl > 63) throw new FHEError('decompBaseLog must be in [1, 63]', FHEErrorCode.INVALID_PARAMETERS);
        const rlk = this._buf(lv * 2 * this._n);
        await this._ctx.evalKeyGenerateAsync(s.buf, bl, lv, this._seed, this._streams(2 * lv), this._std, rlk);
        const prep = this._buf(lv * 2 * this._n);
        await this._ctx.prepareRelinKeyAsync(rlk, prep);
        return this._handle('EvaluationKey', { keyId: sk.keyId, decompBaseLog: bl, decompLevel: lv },
          { buf: rlk, prep, baseLog: bl, level: lv });
      });
    }
    /** BootstrapEngine::generate_bootstrap_key (bootstrap_engine.cpp:308-360)
     *  with a fresh binary LWE key of the parameter set's lweDimension:
     *  GGSW encryptions of its bits (encrypt_ggsw :268-306) and the key
     *  switching key back to it (:367-420).  The LWE key stays with the
     *  secret key's native state (decrypt of bootstrapped ciphertexts). */
    async generateBootstrapKey(sk) {
      this._check();
      return guard(async () => {
        const s = this._st(sk, 'SecretKey');
        const dim = this._params.lweDimension | 0;
        const k = this._params.glweDimension || 1;
        if (dim <= 0) throw new FHEError('parameter set has no LWE dimension (not a TFHE set)', FHEErrorCode.INVALID_PARAMETERS);
        if (k !== 1) throw new FHEError('bootstrapping keys implemented for GLWE dimension 1', FHEErrorCode.INVALID_PARAMETERS);
        const bl = this._params.decompBaseLog > 0 ? this._params.decompBaseLog : 4;
        const lv = this._params.decompLevel > 0 ? this._params.decompLevel : 3;
        const lweDev = this._buf(dim);
        await this._ctx.sampleAsync(SAMPLE.BINARY, this._seed, this._streams(1), 0, lweDev);
        const lweSk = new BigInt64Array(lweDev.download().buffer);
        const n = this._n;
        const bsk = this._buf(dim * 2 * lv * 2 * n);
        await this._ctx.ggswEncryptAsync(lweDev, s.buf, 1, bl, lv, this._seed, this._streams(2), this._std, bsk);
        const bskPrep = this._buf(dim * 2 * lv * 2 * n);
        await this._ctx.prepareGgswAsync(bsk, 1, lv, bskPrep);
        bsk.free();
        const kskA = this._buf(n * lv * dim), kskB = this._buf(n * lv);
        await this._ctx.kskGenerateAsync(s.buf, lweDev, bl, lv, this._seed, this._streams(2), this._std, kskA, kskB);
        s.lweSk = lweSk;
        s.lweDev = lweDev;
        const tp = this._upload(this._identityTestPoly());
        return this._handle('BootstrapKey', { keyId: sk.keyId, lweDimension: dim },
          { buf: bskPrep, bskPrep, kskA, kskB, baseLog: bl, level: lv, ksBaseLog: bl, ksLevel: lv, dim, testPoly: tp });
      });
    }
    /** init_default_test_poly (bootstrap_engine.cpp:57-77) */
    _identityTestPoly() {
      const n = BigInt(this._n), c = new BigUint64Array(this._n);
      for (let i = 0n; i < n; i++) c[Number(i)] = ((((i * this._tEff) / (2n * n)) * this._delta) & M64) % this._q;
      return c;
    }
    /** create_lookup_table (:725-758) over a table f[v], v < lut.length */
    _lutPoly(lut) {
      const n = BigInt(this._n), inMod = BigInt(lut.length), outMod = this._tEff, dOut = this._q / outMod;
      const c = new BigUint64Array(this._n);
      for (let i = 0n; i < n; i++) {
        const v = ((i * inMod + n) / (2n * n)) % inMod;
        c[Number(i)] = (((BigInt(lut[Number(v)]) % outMod) * dOut) & M64) % this._q;
      }
      return c;
    }

    /** KeyManager::generate_threshold_keys (key_manager.cpp:479-560): Shamir
     *  shares s_i = sum_j coeff_j i^j of a fresh ternary master key
     *  (coefficients j >= 1 uniform), computed on the device. */
    async generateThresholdKeys(config) {
      this._check();
      return guard(async () => {
        const t = config && config.threshold | 0, total = config && config.totalShares | 0;
        if (t <= 0 || t > total) throw new FHEError('Invalid threshold parameters', FHEErrorCode.INVALID_PARAMETERS);
        const master = await this.generateSecretKey();
        const ms = state.get(master);
        const coeffs = [ms.buf];
        for (let j = 1; j < t; j++) {
          const c = this._buf(this._n);
          await this._ctx.sampleAsync(SAMPLE.UNIFORM, this._seed, this._streams(1), 0, c);
          coeffs.push(c);
        }
        const shares = [];
        for (let i = 1; i <= total; i++) {
          const acc = this._buf(this._n), term = this._buf(this._n);
          let pw = 1n;
          for (let j = 0; j < t; j++) {
            await this._ctx.mulScalarAsync(coeffs[j], pw, j === 0 ? acc : term);
            if (j > 0) await this._ctx.addAsync(acc, term, acc);
            pw = (pw * BigInt(i)) % this._q;
          }
          term.free();
          const commitment = new Uint8Array(crypto.createHash('sha256').update(Buffer.from(acc.download().buffer)).digest());
          const h = Object.freeze({ shareId: i, handle: acc.handle, commitment, keyId: master.keyId });
          state.set(h, { engine: this, buf: acc });
          shares.push(h);
        }
        const publicKey = await this.generatePublicKey(master);
        return { shares, publicKey, threshold: t, totalShares: total };
      });
    }
    /** KeyManager::partial_decrypt (:584-601): c1 (*) share */
    async partialDecrypt(ct, share) {
      this._check();
      return guard(async () => {
        const c = this._rlwe(ct);
        const s = share && state.get(share);
        if (!s || s.engine !== this) throw new FHEError('not a key share of this engine', FHEErrorCode.INVALID_PARAMETERS);
        if (share.keyId !== ct.keyId) throw new FHEError('Key share does not match the ciphertext key', FHEErrorCode.KEY_MISMATCH);
        const p = this._buf(this._n);
        await this._ctx.polymulAsync(c.buf.view(this._n, this._n), s.buf, p);
        const w = p.download();
        return { shareId: share.shareId, partialResult: toBigIntArray(w, this._n) };
      });
    }
    /** combine_partial_decryptions (:604-632) with lagrange_coefficient
     *  (:566-582), then c0 - sum and decode (decode_packed :150-163) */
    async combinePartialDecryptions(ct, partials, t) {
      this._check();
      return guard(async () => {
        const c = this._rlwe(ct);
        if (!Array.isArray(partials) || partials.length < t) {
          throw new FHEError(`Need ${t} partials, got ${partials ? partials.length : 0}`, FHEErrorCode.THRESHOLD_NOT_MET);
        }
        const q = this._q, idx = partials.map((p) => BigInt(p.shareId));
        const acc = this._buf(this._n), term = this._buf(this._n), pb = this._buf(this._n);
        for (let i = 0; i < partials.length && i < t; i++) {
          let num = 1n, den = 1n;
          for (const j of idx) {
            if (j === idx[i]) continue;
            num = (num * j) % q;
            den = (den * (((j - idx[i]) % q + q) % q)) % q;
          }
          const lambda = (num * modPow(den, q - 2n, q)) % q;
          pb.upload(BigUint64Array.from(partials[i].partialResult.map((x) => u64(x))));
          await this._ctx.mulScalarAsync(pb, lambda, i === 0 ? acc : term);
          if (i > 0) await this._ctx.addAsync(acc, term, acc);
        }
        await this._ctx.subAsync(c.buf.view(0, this._n), acc, acc);
        const phase = acc.download();
        const vals = new BigUint64Array(this._n);
        for (let i = 0; i < this._n; i++) vals[i] = ((phase[i] * this._tEff + q / 2n) / q) % this._tEff;
        return this._decryptionResult(vals, null, c.packed);
      });
    }

    // ---- encrypt / decrypt (encryption.cpp:171-348)
    async encrypt(plaintext, pk) {
      this._check();
      return guard(async () => {
        const p = this._st(pk, 'PublicKey');
        const slots = this._slots(plaintext);
        const ct = this._buf(2 * this._n);
        await this._ctx.encryptSampledAsync(this._t, p.prep, this._upload(slots), this._seed, this._streams(3), this._std, ct);
        return { ciphertext: this._ct(ct, pk.keyId, this._initialBudget, 1, { packed: !!(plaintext.isPacked && plaintext.values.length > 1) }) };
      });
    }
    async encryptValue(value, pk) { return (await this.encrypt(this.createPlaintext(value), pk)).ciphertext; }
    async encryptPacked(values, pk) { return (await this.encrypt(this.createPackedPlaintext(values), pk)).ciphertext; }
    async getZeroCiphertext(pk) { return this.encryptValue(0n, pk); }
    /** batch_encrypt (encryption.cpp:460-540): one device launch for the whole batch */
    async batchEncrypt(pts, pk, opts) {
      this._check();
      return guard(async () => {
        const p = this._st(pk, 'PublicKey');
        const start = Date.now(), n = this._n, B = pts.length;
        if (B === 0) return { ciphertexts: [], elapsedMs: 0, throughputPerSecond: 0 };
        const slots = new BigUint64Array(B * n);
        pts.forEach((pt, i) => slots.set(this._slots(pt), i * n));
        const all = this._buf(2 * n * B);
        await this._ctx.encryptSampledAsync(this._t, p.prep, this._upload(slots), this._seed, this._streams(3), this._std, all);
        const ciphertexts = pts.map((pt, i) => this._ct(all.view(2 * n * i, 2 * n), pk.keyId, this._initialBudget, 1,
          { packed: !!(pt.isPacked && pt.values.length > 1) }));
        const ms = Date.now() - start;
        return { ciphertexts, elapsedMs: ms, throughputPerSecond: ms > 0 ? (B * 1000) / ms : 0 };
      });
    }
    _decryptionResult(vals, maxNoise, packed) {
      const budget = maxNoise === null ? this._initialBudget : this._budgetOf(maxNoise);
      const values = packed ? toBigIntArray(vals, this._n) : [vals[0]];
      const r = {
        plaintext: Object.freeze({ __brand: 'Plaintext', values, plaintextModulus: this._tEff, isPacked: !!packed }),
        remainingNoiseBudget: budget,
        success: budget >= 0,
      };
      if (!r.success) r.errorMessage = 'Noise budget exhausted - decryption may be incorrect';
      r._slots = vals;
      return r;
    }
    async _decryptRaw(ct, sk) {
      const c = this._st(ct, 'Ciphertext'), s = this._st(sk, 'SecretKey');
      if (ct.keyId !== sk.keyId) return { mismatch: true };
      if (c.kind === 'lwe') {
        if (!s.lweSk) throw new FHEError('no LWE key: generateBootstrapKey(sk) was not called', FHEErrorCode.INVALID_PARAMETERS);
        const v = this._buf(1), ph = this._buf(1);
        await this._ctx.lweDecryptAsync(this._t, s.lweDev, c.buf.view(0, c.dim), c.buf.view(c.dim, 1), v, ph);
        const phase = ph.download()[0];
        // the LWE noise: distance of the phase to round(p t / q) delta (compute_noise_budget's measure)
        const r = ((phase * this._tEff + this._q / 2n) / this._q);
        const exp = ((r * this._delta) & M64) % this._q;
        let d = phase >= exp ? phase - exp : exp - phase;
        if (d > this._q / 2n) d = this._q - d;
        const vals = new BigUint64Array(this._n);
        vals[0] = v.download()[0];
        return { vals, maxNoise: d, packed: false };
      }
      const vals = this._buf(this._n), mx = this._buf(1);
      await this._ctx.decryptAsync(this._t, s.prep, c.buf, c.comps, ct.isNtt ? 1 : 0, vals, mx);
      return { vals: vals.download(), maxNoise: mx.download()[0], packed: c.packed };
    }
    async decrypt(ct, sk) {
      this._check();
      return guard(async () => {
        const r = await this._decryptRaw(ct, sk);
        if (r.mismatch) {
          return { plaintext: Object.freeze({ __brand: 'Plaintext', values: [], plaintextModulus: this._tEff, isPacked: false }),
            remainingNoiseBudget: 0, success: false,
            errorMessage: 'Key ID mismatch: ciphertext was encrypted with different key' };
        }
        return this._decryptionResult(r.vals, r.maxNoise, r.packed);
      });
    }
    async decryptValue(ct, sk) {
      const r = await this.decrypt(ct, sk);
      if (!r.success) throw new FHEError(r.errorMessage || 'Decryption failed', FHEErrorCode.NOISE_BUDGET_EXHAUSTED);
      return r.plaintext.values.length ? r.plaintext.values[0] : 0n;
    }
    async decryptPacked(ct, sk, numValues) {
      const r = await this.decrypt(ct, sk);
      if (!r.success) throw new FHEError(r.errorMessage || 'Decryption failed', FHEErrorCode.NOISE_BUDGET_EXHAUSTED);
      return toBigIntArray(r._slots, Math.min(numValues, this._n));
    }
    async getNoiseBudget(ct, sk) {
      this._check();
      return guard(async () => {
        const r = await this._decryptRaw(ct, sk);
        if (r.mismatch) throw new FHEError('Key ID mismatch', FHEErrorCode.KEY_MISMATCH);
        return this._budgetOf(r.maxNoise);
      });
    }
    /** estimate_noise_budget (:446-450): the tracked estimate */
    estimateNoiseBudget(ct) {
      this._check();
      this._st(ct, 'Ciphertext');
      return ct.noiseBudget;
    }

    // ---- additive operations (encryption.cpp:594-735)
    async _addsub(ct1, ct2, sub) {
      this._check();
      return guard(async () => {
        const a = this._rlwe(ct1), b = this._rlwe(ct2);
        this._sameKey(ct1, ct2, sub ? 'subtract' : 'add');
        if (ct1.isNtt !== ct2.isNtt) throw new FHEError('Cannot combine ciphertexts in different representations (NTT vs coefficient)', FHEErrorCode.INVALID_PARAMETERS);
        if (a.comps !== b.comps) throw new FHEError('ciphertext degrees differ', FHEErrorCode.INVALID_PARAMETERS);
        const out = this._buf(a.comps * this._n);
        await (sub ? this._ctx.subAsync(a.buf, b.buf, out) : this._ctx.addAsync(a.buf, b.buf, out));
        return this._ct(out, ct1.keyId, Math.min(ct1.noiseBudget, ct2.noiseBudget) - 1, ct1.degree,
          { packed: a.packed || b.packed });
      });
    }
    async add(ct1, ct2) { return this._addsub(ct1, ct2, false); }
    async subtract(ct1, ct2) { return this._addsub(ct1, ct2, true); }
    async negate(ct) {
      this._check();
      return guard(async () => {
        const a = this._rlwe(ct);
        const out = this._buf(a.comps * this._n);
        await this._ctx.negateAsync(a.buf, out);
        return this._ct(out, ct.keyId, ct.noiseBudget, ct.degree, { packed: a.packed });
      });
    }
    /** add_plain (:638-665): c0 + encode(pt), the rest copied; budget - 0.5 */
    async addPlain(ct, pt) {
      this._check();
      return guard(async () => {
        const a = this._rlwe(ct), n = this._n;
        const out = this._buf(a.comps * n);
        await this._ctx.addPlainAsync(this._t, a.buf.view(0, 2 * n), this._upload(this._slots(pt)), ct.isNtt ? 1 : 0,
          out.view(0, 2 * n));
        if (a.comps === 3) out.copyFrom(a.buf, 2 * n, 2 * n, n);
        return this._ct(out, ct.keyId, ct.noiseBudget - 0.5, ct.degree,
          { packed: a.packed || !!(pt.isPacked && pt.values.length > 1) });
      });
    }
    /** add_scalar (:685-688) */
    async addScalar(ct, value) { return this.addPlain(ct, this.createPlaintext(value)); }
    async batchAdd(cts, progress) {
      this._check();
      if (!Array.isArray(cts) || cts.length === 0) throw new FHEError('Empty array', FHEErrorCode.INVALID_PARAMETERS);
      const start = Date.now();
      let r = cts[0];
      for (let i = 1; i < cts.length; i++) {
        r = await this.add(r, cts[i]);
        if (progress) {
          progress({ stage: 'batch_add', current: i + 1, total: cts.length, elapsedMs: Date.now() - start,
            progressPercent: ((i + 1) / cts.length) * 100 });
        }
      }
      return r;
    }

    // ---- multiplicative operations (encryption.cpp:737-980)
    async multiply(ct1, ct2) {
      this._check();
      return guard(async () => {
        const a = this._rlwe(ct1), b = this._rlwe(ct2);
        this._sameKey(ct1, ct2, 'multiply');
        if (a.comps !== 2 || b.comps !== 2) throw new FHEError('multiply takes degree-1 ciphertexts (relinearize first)', FHEErrorCode.INVALID_PARAMETERS);
        const out = this._buf(3 * this._n);
        await this._ctx.ctMultiplyAsync(a.buf, b.buf, out, ct1.isNtt ? 1 : 0);
        const red = Math.log2(this._n) + 5;
        return this._ct(out, ct1.keyId, Math.min(ct1.noiseBudget, ct2.noiseBudget) - red, 2,
          { packed: a.packed || b.packed });
      });
    }
    async relinearize(ct, ek) {
      this._check();
      return guard(async () => {
        const a = this._rlwe(ct);
        if (a.comps === 2) {  // already degree 1: a copy (:906-909)
          const out = this._buf(2 * this._n);
          out.copyFrom(a.buf);
          return this._ct(out, ct.keyId, ct.noiseBudget, 1, { packed: a.packed });
        }
        const e = this._st(ek, 'EvaluationKey');
        if (ct.keyId !== ek.keyId) throw new FHEError('Evaluation key does not match ciphertext key', FHEErrorCode.KEY_MISMATCH);
        const out = this._buf(2 * this._n);
        await this._ctx.relinearizePreparedAsync(a.buf, e.prep, e.baseLog, out);
        return this._ct(out, ct.keyId, ct.noiseBudget - 1, 1, { packed: a.packed });
      });
    }
    async multiplyRelin(ct1, ct2, ek) { return this.relinearize(await this.multiply(ct1, ct2), ek); }
    async square(ct) { return this.multiply(ct, ct); }
    async squareRelin(ct, ek) { return this.relinearize(await this.square(ct), ek); }
    /** multiply_plain (:809-848): each component times encode(pt); budget - 2 */
    async multiplyPlain(ct, pt) {
      this._check();
      return guard(async () => {
        const a = this._rlwe(ct), n = this._n;
        const enc = this._encoded(pt);
        const rep = this._buf(a.comps * n);
        for (let c = 0; c < a.comps; c++) rep.upload(enc, c * n);
        const out = this._buf(a.comps * n);
        await this._ctx.polymulAsync(a.buf, rep, out);
        return this._ct(out, ct.keyId, ct.noiseBudget - 2, ct.degree, { packed: a.packed });
      });
    }
    /** multiply_scalar (:890-903): budget - 1 */
    async multiplyScalar(ct, scalar) {
      this._check();
      return guard(async () => {
        const a = this._rlwe(ct);
        const out = this._buf(a.comps * this._n);
        await this._ctx.mulScalarAsync(a.buf, u64(scalar), out);
        return this._ct(out, ct.keyId, ct.noiseBudget - 1, ct.degree, { packed: a.packed });
      });
    }

    // ---- bootstrapping (bootstrap_engine.cpp:676-758)
    async _bootstrap(ct, bk, testPoly) {
      const b = this._st(bk, 'BootstrapKey');
      const c = this._st(ct, 'Ciphertext');
      if (ct.keyId !== bk.keyId) throw new FHEError('Bootstrap key does not match the ciphertext key', FHEErrorCode.KEY_MISMATCH);
      const n = this._n, dim = b.dim;
      let la, lb;
      if (c.kind === 'lwe') {
        la = c.buf.view(0, dim);
        lb = c.buf.view(dim, 1);
      } else {
        if (c.comps !== 2) throw new FHEError('bootstrap takes degree-1 ciphertexts', FHEErrorCode.INVALID_PARAMETERS);
        // RLWE (c0, c1) is the GLWE (mask c1, body c0): sample_extract
        // (:594-624) of coefficient 0, then key_switch (:626-674) to the LWE key
        const glwe = this._buf(2 * n);
        glwe.copyFrom(c.buf, 0, n, n);
        glwe.copyFrom(c.buf, n, 0, n);
        const ea = this._buf(n), eb = this._buf(1);
        await this._ctx.sampleExtractAsync(1, glwe, ea, eb);
        la = this._buf(dim);
        lb = this._buf(1);
        await this._ctx.keySwitchAsync(b.ksBaseLog, b.ksLevel, b.kskA, b.kskB, ea, eb, la, lb);
      }
      const out = this._buf(dim + 1);
      await this._ctx.bootstrapPreparedAsync(la, lb, b.bskPrep, testPoly, b.kskA, b.kskB, b.baseLog, b.level,
        b.ksBaseLog, b.ksLevel, out.view(0, dim), out.view(dim, 1));
      return this._handle('Ciphertext', { keyId: ct.keyId, noiseBudget: this._params.noiseBudget, isNtt: false, degree: 1 },
        { buf: out, kind: 'lwe', comps: 0, dim, packed: false });
    }
    async bootstrap(ct, bk) {
      this._check();
      return guard(async () => this._bootstrap(ct, bk, this._st(bk, 'BootstrapKey').testPoly));
    }
    async programmableBootstrap(ct, bk, lut) {
      this._check();
      return guard(async () => {
        if (!Array.isArray(lut) || lut.length === 0) throw new FHEError('lut must be a non-empty bigint[]', FHEErrorCode.INVALID_PARAMETERS);
        return this._bootstrap(ct, bk, this._upload(this._lutPoly(lut)));
      });
    }

    // ---- serialisation: binary = header words + the native words, checksum = SHA-256
    _serialize(kind, h, words, meta, opts) {
      const fmt = (opts && opts.format) || 'binary';
      const head = [BigInt(SERIAL_MAGIC), 1n, BigInt(KINDS.indexOf(kind)), BigInt(this._n), this._q, BigInt(h.keyId)];
      const metaJson = Buffer.from(JSON.stringify(meta, (k, v) => (typeof v === 'bigint' ? v.toString() : v)));
      const hw = BigUint64Array.from(head);
      let data = Buffer.concat([Buffer.from(hw.buffer), Buffer.from(new Uint32Array([metaJson.length]).buffer), metaJson,
        Buffer.from(words.buffer, words.byteOffset, words.byteLength)]);
      if (fmt === 'json') {
        data = Buffer.from(JSON.stringify({ head: head.map(String), meta: metaJson.toString(),
          words: Buffer.from(words.buffer, words.byteOffset, words.byteLength).toString('base64') }));
      } else if (fmt === 'compressed') {
        data = zlib.deflateSync(data);
      } else if (fmt !== 'binary') {
        throw new FHEError(`unknown format ${fmt}`, FHEErrorCode.SERIALIZATION_ERROR);
      }
      return { data: new Uint8Array(data), format: fmt, checksum: new Uint8Array(crypto.createHash('sha256').update(data).digest()) };
    }
    _parse(s, kind) {
      if (!s || !s.data) throw new FHEError('no serialized data', FHEErrorCode.SERIALIZATION_ERROR);
      const data = Buffer.from(s.data);
      const sum = crypto.createHash('sha256').update(data).digest();
      if (s.checksum && !sum.equals(Buffer.from(s.checksum))) throw new FHEError('checksum mismatch', FHEErrorCode.SERIALIZATION_ERROR);
      try {
        let head, meta, words;
        if (s.format === 'json') {
          const j = JSON.parse(data.toString());
          head = j.head.map(BigInt);
          meta = JSON.parse(j.meta);
          const w = Buffer.from(j.words, 'base64');
          words = new BigUint64Array(w.buffer.slice(w.byteOffset, w.byteOffset + w.length));
        } else {
          const raw = s.format === 'compressed' ? zlib.inflateSync(data) : data;
          const b = Buffer.from(raw);
          const hw = new BigUint64Array(b.buffer.slice(b.byteOffset, b.byteOffset + 48));
          head = Array.from(hw);
          const ml = b.readUInt32LE(48);
          meta = JSON.parse(b.slice(52, 52 + ml).toString());
          const wb = b.slice(52 + ml);
          words = new BigUint64Array(wb.buffer.slice(wb.byteOffset, wb.byteOffset + wb.length));
        }
        if (head[0] !== BigInt(SERIAL_MAGIC) || head[1] !== 1n || KINDS[Number(head[2])] !== kind) throw new Error('header');
        if (head[3] !== BigInt(this._n) || head[4] !== this._q) throw new Error('parameters differ from this engine');
        return { keyId: head[5], meta, words };
      } catch (e) {
        throw new FHEError(`malformed ${kind} data: ${e.message}`, FHEErrorCode.SERIALIZATION_ERROR);
      }
    }
    async serializeSecretKey(sk, opts) {
      this._check();
      const s = this._st(sk, 'SecretKey');
      const r = this._serialize('secret', sk, s.buf.download(), { lweSk: s.lweSk ? Array.from(s.lweSk, String) : null }, opts);
      return Object.assign(r, { keyType: 'secret', version: 1 });
    }
    async deserializeSecretKey(data) {
      this._check();
      return guard(async () => {
        const { keyId, meta, words } = this._parse(data, 'secret');
        const buf = this._upload(words), prep = this._buf(2 * this._n);
        await this._ctx.prepareSecretKeyAsync(buf, prep);
        const st = { buf, prep };
        if (meta.lweSk) {
          st.lweSk = BigInt64Array.from(meta.lweSk.map(BigInt));
          st.lweDev = this._upload(st.lweSk);
        }
        return this._handle('SecretKey', { keyId }, st);
      });
    }
    async serializePublicKey(pk, opts) {
      this._check();
      const s = this._st(pk, 'PublicKey');
      return Object.assign(this._serialize('public', pk, s.buf.download(), {}, opts), { keyType: 'public', version: 1 });
    }
    async deserializePublicKey(data) {
      this._check();
      return guard(async () => {
        const { keyId, words } = this._parse(data, 'public');
        const buf = this._upload(words), prep = this._buf(2 * this._n);
        await this._ctx.preparePublicKeyAsync(buf, prep);
        return this._handle('PublicKey', { keyId }, { buf, prep });
      });
    }
    async serializeCiphertext(ct, opts) {
      this._check();
      const c = this._st(ct, 'Ciphertext');
      const meta = { noiseBudget: ct.noiseBudget, isNtt: ct.isNtt, degree: ct.degree, kind: c.kind, comps: c.comps,
        dim: c.dim || 0, packed: c.packed };
      const r = this._serialize('ciphertext', ct, c.buf.download(), meta, opts);
      return Object.assign(r, { keyId: ct.keyId, version: 1 });
    }
    async deserializeCiphertext(data) {
      this._check();
      return guard(async () => {
        const { keyId, meta, words } = this._parse(data, 'ciphertext');
        return this._handle('Ciphertext', { keyId, noiseBudget: meta.noiseBudget, isNtt: meta.isNtt, degree: meta.degree },
          { buf: this._upload(words), kind: meta.kind, comps: meta.comps, dim: meta.dim, packed: meta.packed });
      });
    }

    // ---- plaintexts and introspection
    createPlaintext(value) {
      this._check();
      return Object.freeze({ __brand: 'Plaintext', values: [BigInt(value)], plaintextModulus: this._tEff, isPacked: false });
    }
    createPackedPlaintext(values) {
      this._check();
      return Object.freeze({ __brand: 'Plaintext', values: values.map((v) => BigInt(v)), plaintextModulus: this._tEff, isPacked: true });
    }
    getParams() { this._check(); return this._params; }
    getHardwareCapabilities() {
      this._check();
      const hw = native.detectHardware();
      return { hasSme: false, hasMetal: false, hasNeon: false, hasAmx: false, hasNeuralEngine: false, metalGpuCores: 0,
        unifiedMemorySize: 0n, hasHip: hw.hasHip, gpuDevices: hw.gpuDevices, computeUnits: hw.computeUnits,
        hbmBytes: BigInt(hw.hbmBytes), arch: hw.arch, deviceName: hw.deviceName };
    }
    getSlotCount() { this._check(); return this._n; }
    /** the native context (NttContext) for batched array-level work */
    get context() { return this._ctx; }
    /** the DeviceBuffer behind a handle (advanced use: batched kernels) */
    deviceBuffer(h) { const s = h && state.get(h); return s ? s.buf : undefined; }
    dispose() {
      if (!this._disposed) {
        this._disposed = true;
        this._ctx = null;
      }
    }
  }

  async function createEngine(params, options) {
    const p = createParameterSet(params);
    try {
      return new FHEEngineImpl(p, options);
    } catch (e) {
      throw toFHEError(e);
    }
  }
  return { FHEEngineImpl, createEngine };
}

/**
 * Context defaults from the environment (SURVEY.md section 5 config flags):
 * FHE_NTT_MODE = compat | negacyclic when no mode is given; FHE_GPU_DEVICES
 * = comma-separated GPU ordinals when neither device nor devices is given
 * (one entry: that device; several: a multi-device context).
 */
function envDefaults({ mode, device, devices } = {}) {
  if (mode === undefined) mode = (process.env.FHE_NTT_MODE || 'compat').trim() || 'compat';
  if (device === undefined && devices === undefined && process.env.FHE_GPU_DEVICES) {
    const list = process.env.FHE_GPU_DEVICES.split(',').filter((x) => x.trim() !== '').map(Number);
    if (list.some((d) => !Number.isInteger(d) || d < 0)) {
      throw new RangeError(`FHE_GPU_DEVICES must be a comma-separated list of ordinals, got ${process.env.FHE_GPU_DEVICES}`);
    }
    if (list.length === 1) device = list[0];
    else if (list.length > 1) devices = list;
  }
  if (device === undefined) device = devices ? devices[0] : 0;
  return { mode, device, devices };
}

module.exports = {
  envDefaults, FHEError, FHEErrorCode, NTT_PRIMES, calculateDerivedParameters, createParameterSet, getAvailablePresets,
  makeEngineClass, toFHEError,
};
