'use strict';
// Node-side tests of the N-API addon (node:assert; there is no vitest here).
// Mirrors the reference's JS-visible contract (index.d.ts, src/native/lib.rs)
// and, in "gpu" mode, checks the batched engine against the golden fixtures.
//   node tests/js/napi_test.js [cpu|gpu]
const assert = require('assert');
const fs = require('fs');
const path = require('path');

const ROOT = path.join(__dirname, '..', '..');
const fhe = require(path.join(ROOT, 'node-fhe-accelerate_amd', 'lib'));
const mode = process.argv[2] || 'cpu';
const golden = (name) => JSON.parse(fs.readFileSync(path.join(ROOT, 'tests', 'golden', name), 'utf8'),
  // keep big integers exact: JSON numbers above 2^53 are parsed from text
  undefined);
const goldenBig = (name) => {
  const txt = fs.readFileSync(path.join(ROOT, 'tests', 'golden', name), 'utf8');
  return JSON.parse(txt.replace(/([\[:,])(\d{16,})(?=[,\]}])/g, '$1"$2"'));
};
const U = (xs) => BigUint64Array.from(xs.map((x) => BigInt(x)));

let passed = 0;
const asyncTests = [];
function test(name, fn) {
  fn();
  passed += 1;
  console.log('ok -', name);
}

test('exports match index.d.ts', () => {
  for (const k of ['initialize', 'detectHardware', 'version', 'ModularArithmetic']) {
    assert.ok(k in fhe, k);
  }
  fhe.initialize();
  assert.ok(fhe.version().length > 0);
  const hw = fhe.detectHardware();
  for (const k of ['hasSme', 'hasMetal', 'hasNeon', 'hasAmx', 'metalGpuCores', 'unifiedMemorySize']) {
    assert.ok(k in hw, k);
  }
  assert.strictEqual(typeof hw.hasHip, 'boolean');
});

test('ModularArithmetic semantics (modular_arithmetic.cpp:52-165)', () => {
  const q = 132120577;
  const m = new fhe.ModularArithmetic(q);
  assert.strictEqual(m.getModulus(), q);
  assert.strictEqual(m.modAdd(q - 1, 5), 4);
  assert.strictEqual(m.modSub(3, 5), q - 2);
  // fromMontgomery(toMontgomery(a)) with the reference's constants
  const k = golden('reference_kat.json');
  assert.ok(k.psi_table.length === 4);
  assert.throws(() => new fhe.ModularArithmetic(0), /Modulus must be positive/);
  assert.throws(() => new fhe.ModularArithmetic(96), /odd and non-zero/);
  assert.throws(() => m.montgomeryMul(-1, 2), /Inputs must be non-negative/);
  assert.throws(() => m.toMontgomery(-1), /Input must be non-negative/);
});

if (mode === 'cpu') {
  test('compute without a GPU fails loudly (no CPU fallback)', () => {
    const hw = fhe.detectHardware();
    if (hw.gpuDevices > 0) return;
    assert.throws(() => new fhe.PolynomialEngine(1024, 132120577), /no HIP device/);
    assert.throws(() => fhe.modmulBatch(17n, U([1]), U([2]), new BigUint64Array(1)), /no HIP device/);
  });
  test('parameter validation messages', () => {
    assert.throws(() => new fhe.NttContext(12, 97n), /power of 2/);
    assert.throws(() => new fhe.NttContext(8, 96n), /Modulus must be odd/);
    assert.throws(() => new fhe.NttContext(16, 17n), /NTT-friendly/);
  });
} else {
  test('forward/inverse/polymul vs golden fixtures', () => {
    for (const c of goldenBig('ntt_small.json')) {
      const e = new fhe.PolynomialEngine(c.n, BigInt(c.q));
      assert.strictEqual(e.info().primitiveRoot, BigInt(c.psi));
      const x = U(c.x);
      const f = e.toNtt(x.slice());
      assert.deepStrictEqual(Array.from(f), c.forward.map(BigInt), `forward n=${c.n}`);
      assert.deepStrictEqual(Array.from(e.fromNtt(x.slice())), c.inverse.map(BigInt), `inverse n=${c.n}`);
      assert.deepStrictEqual(Array.from(e.multiply(x, U(c.y))), c.polymul.map(BigInt), `polymul n=${c.n}`);
      assert.deepStrictEqual(Array.from(e.forwardMultiply(x, U(c.w))), c.fwd_mul.map(BigInt));
      assert.deepStrictEqual(Array.from(e.fromNtt(f)), c.x.map(BigInt), 'round trip');
    }
  });
  test('modmulBatch vs golden', () => {
    for (const c of goldenBig('modmul.json')) {
      const out = new BigUint64Array(c.a.length);
      fhe.modmulBatch(BigInt(c.q), U(c.a), U(c.b), out);
      assert.deepStrictEqual(Array.from(out), c.c.map(BigInt), `q=${c.q}`);
    }
  });
  test('mlMontgomeryMulBatch vs golden', () => {
    for (const c of goldenBig('multi_limb.json')) {
      const out = new BigUint64Array(c.a.length);
      fhe.mlMontgomeryMulBatch(U(c.q), U(c.a), U(c.b), out);
      assert.deepStrictEqual(Array.from(out), c.c.map(BigInt));
    }
  });
  test('externalProduct vs golden', () => {
    for (const c of goldenBig('extprod.json')) {
      const e = new fhe.PolynomialEngine(c.n, BigInt(c.q));
      const out = e.externalProduct(U(c.glwe), U(c.ggsw), c.base_log, c.level);
      assert.deepStrictEqual(Array.from(out), c.out.map(BigInt));
    }
  });
  test('ciphertext multiply / relinearize / blind rotate vs golden', () => {
    for (const c of goldenBig('cipher.json')) {
      const e = new fhe.PolynomialEngine(c.n, BigInt(c.q));
      let got;
      if (c.op === 'ct_multiply') got = e.ctMultiply(U(c.ct1), U(c.ct2));
      else if (c.op === 'relinearize') got = e.relinearize(U(c.ct3), U(c.rlk), c.base_log);
      else {
        got = U(c.acc);
        e.blindRotate(got, U(c.lwe_a), U([c.lwe_b]), U(c.bsk), c.base_log, c.level);
        assert.strictEqual(typeof e.brRepairCount(), 'number');
      }
      assert.deepStrictEqual(Array.from(got), c.out.map(BigInt), `${c.op} n=${c.n}`);
    }
  });
  test('createEngine: ciphertext multiply / relinearize vs golden (async FHEEngine surface)', () => {
    const pending = [];
    for (const c of goldenBig('cipher.json')) {
      if (c.op === 'blind_rotate') continue;
      const custom = { polyDegree: c.n, moduli: [BigInt(c.q)], decompBaseLog: c.base_log || 4 };
      pending.push(Promise.resolve(new fhe.GpuFHEEngine(custom)).then(async (eng) => {
        const got = c.op === 'ct_multiply' ? await eng.multiply(U(c.ct1), U(c.ct2))
          : await eng.relinearize(U(c.ct3), U(c.rlk), c.base_log);
        assert.deepStrictEqual(Array.from(got), c.out.map(BigInt), `${c.op} n=${c.n}`);
      }));
    }
    asyncTests.push(Promise.all(pending));
  });
  // splitmix64(seed ^ i) % q (oracle_splitmix_fill) -- regenerates the seeded fixture inputs
  const M64 = (1n << 64n) - 1n;
  const splitmix = (seed, q, count) => {
    const out = new BigUint64Array(count);
    for (let i = 0; i < count; i++) {
      let x = (BigInt(seed) ^ BigInt(i)) & M64;
      x = (x + 0x9E3779B97F4A7C15n) & M64;
      x = ((x ^ (x >> 30n)) * 0xBF58476D1CE4E5B9n) & M64;
      x = ((x ^ (x >> 27n)) * 0x94D049BB133111EBn) & M64;
      x ^= x >> 31n;
      out[i] = q ? x % BigInt(q) : x;
    }
    return out;
  };
  const ternary = (seed, q, n) => splitmix(seed, 3, n).map((v) => (v === 2n ? BigInt(q) - 1n : v));
  const small = (seed, q, n) => splitmix(seed, 7, n).map((v) => (v < 3n ? BigInt(q) + v - 3n : v - 3n));
  const sha = (a) => require('crypto').createHash('sha256').update(Buffer.from(a.buffer, a.byteOffset, a.byteLength))
    .digest('hex');
  test('engine encrypt / decrypt / addPlain vs golden (async forms)', () => {
    const pending = [];
    for (const c of goldenBig('engine.json')) {
      if (c.op !== 'engine') continue;
      const eng = new fhe.GpuFHEEngine({ polyDegree: c.n, moduli: [BigInt(c.q)], plaintextModulus: c.t });
      pending.push((async () => {
        const pk = await eng.importPublicKey(U(c.pk.slice(0, c.n)), U(c.pk.slice(c.n)));
        const sk = await eng.importSecretKey(U(c.sk));
        const ct = await eng.encrypt(U(c.values), pk, { u: U(c.u), e1: U(c.e1), e2: U(c.e2) });
        assert.deepStrictEqual(Array.from(ct), c.ct.map(BigInt), `encrypt n=${c.n}`);
        const d = await eng.decrypt(ct, sk, { phase: true });
        assert.deepStrictEqual(Array.from(d.values), c.dec.map(BigInt), `decrypt n=${c.n}`);
        assert.deepStrictEqual(Array.from(d.phase), c.phase.map(BigInt));
        assert.strictEqual(d.maxNoise[0], BigInt(c.max_noise));
        const ap = await eng.addPlain(ct, U(c.values));
        assert.deepStrictEqual(Array.from(ap), c.add_plain.map(BigInt), `addPlain n=${c.n}`);
      })());
    }
    asyncTests.push(Promise.all(pending));
  });
  test("GpuFHEEngine (array level) bfv-128-simd: encrypt -> multiply -> relinearize -> decrypt vs golden", () => {
    const c = goldenBig('engine.json').find((x) => x.op === 'bfv_flow');
    asyncTests.push(Promise.resolve(new fhe.GpuFHEEngine(fhe.PRESETS[c.preset])).then(async (eng) => {
      const n = c.n, q = BigInt(c.q), S = c.seeds;
      assert.strictEqual(eng.getSlotCount(), n);
      assert.strictEqual(eng.q, q);
      const sk = await eng.importSecretKey(ternary(S.sk, q, n));
      const pk = await eng.generatePublicKey(sk, { a: splitmix(S.a, q, n), e: small(S.e_pk, q, n) });
      assert.strictEqual(sha(pk.poly), c.sha_pk, 'public key');
      const cts = [];
      for (let j = 0; j < 2; j++) {
        cts.push(await eng.encrypt(splitmix(S.values[j], eng.t, n), pk,
          { u: ternary(S.u[j], q, n), e1: small(S.e1[j], q, n), e2: small(S.e2[j], q, n) }));
      }
      assert.strictEqual(sha(cts[0]), c.sha_ct0, 'encrypt 0');
      assert.strictEqual(sha(cts[1]), c.sha_ct1, 'encrypt 1');
      const ct3 = await eng.multiply(cts[0], cts[1]);
      assert.strictEqual(sha(ct3), c.sha_ct3, 'multiply');
      const ek = await eng.generateEvalKey(sk, c.base_log,
        { level: c.level, a: S.rlk_a.map((s) => splitmix(s, q, n)), e: S.rlk_e.map((s) => small(s, q, n)) });
      assert.strictEqual(ek.level, c.level);
      assert.strictEqual(sha(ek.rlk), c.sha_rlk, 'evaluation key');
      const rel = await eng.relinearize(ct3, ek);
      assert.strictEqual(sha(rel), c.sha_relin, 'relinearize');
      const d = await eng.decrypt(rel, sk);
      assert.strictEqual(sha(d.values), c.sha_dec, 'decrypt');
      assert.strictEqual(d.maxNoise[0], BigInt(c.max_noise));
      const d0 = await eng.decrypt(cts[0], sk);
      assert.strictEqual(sha(d0.values), c.sha_dec_ct0);
      assert.strictEqual(d0.maxNoise[0], BigInt(c.max_noise_ct0));
      // the promise-returning forms run off the JS thread: the event loop
      // turns (setImmediate callbacks run) while they are in flight
      let ticks = 0, on = true;
      const spin = () => { ticks += 1; if (on) setImmediate(spin); };
      setImmediate(spin);
      const before = ticks;
      await Promise.all([eng.multiply(cts[0], cts[1]), eng.multiply(cts[1], cts[0]), eng.decrypt(cts[1], sk)]);
      on = false;
      assert.ok(ticks > before, 'event loop blocked while the async calls ran');
    }));
  });
  test('concurrent async jobs on one N=32768 context (big-N scratch) vs golden', () => {
    // forwardAsync and ctMultiplyAsync queued together on one NttContext:
    // both stage host arrays through the context's big-N scratch
    // (two-pass transforms, BigSync) and must not disturb each other
    const c = goldenBig('ntt_large.json').find((x) => x.n === 32768 && BigInt(x.q) === 132120577n);
    const n = c.n, q = BigInt(c.q);
    const ctx = new fhe.NttContext(n, q);
    const x = splitmix(c.seed_x, q, 4 * n), y = splitmix(c.seed_y, q, 4 * n);
    const fx = x.slice();
    const ct = new BigUint64Array(6 * n);
    const fy = y.slice();
    asyncTests.push(Promise.all([ctx.forwardAsync(fx), ctx.ctMultiplyAsync(x, y, ct), ctx.forwardAsync(fy)])
      .then(() => {
        assert.strictEqual(sha(fx), c.sha_forward, 'forward');
        assert.strictEqual(sha(ct), c.sha_ct_multiply, 'ct multiply');
        const fy2 = y.slice();
        ctx.forward(fy2);
        assert.deepStrictEqual(Array.from(fy), Array.from(fy2), 'second forward');
      }));
  });
  test('DeviceBuffer freed while an async job that reads it is queued', () => {
    // the job pins the block: the freed input must not be handed to the
    // next allocation (and overwritten) before the queued job has read it
    const c = goldenBig('ntt_large.json').find((x) => x.n === 16384 && BigInt(x.q) === 132120577n);
    const n = c.n, q = BigInt(c.q);
    const ctx = new fhe.NttContext(n, q);
    const x = splitmix(c.seed_x, q, 4 * n);
    const outs = [], pending = [];
    for (let r = 0; r < 4; r++) {
      const a = new fhe.DeviceBuffer(ctx, 4 * n).upload(x);
      const out = new fhe.DeviceBuffer(ctx, 4 * n);
      pending.push(ctx.forwardAsync(a, out));
      a.free();
      new fhe.DeviceBuffer(ctx, 4 * n).upload(new BigUint64Array(4 * n));  // would reuse a's memory
      outs.push(out);
    }
    asyncTests.push(Promise.all(pending).then(() => {
      for (const o of outs) assert.strictEqual(sha(o.download()), c.sha_forward);
    }));
  });
  test('multi-device NttContext splits host batches', () => {
    const hw = fhe.detectHardware();
    const devs = hw.gpuDevices > 1 ? [0, 1] : [0, 0];
    const c = goldenBig('ntt_small.json').find((x) => x.n === 1024);
    const ctx = new fhe.NttContext(c.n, BigInt(c.q), 0, devs);
    assert.strictEqual(ctx.info().devices, 2);
    const x = U(c.x);
    const two = new BigUint64Array(2 * c.n);
    two.set(x, 0);
    two.set(x, c.n);
    ctx.forward(two);
    assert.deepStrictEqual(Array.from(two.slice(c.n)), c.forward.map(BigInt));
    assert.deepStrictEqual(Array.from(two.slice(0, c.n)), c.forward.map(BigInt));
  });
  test('negacyclic mode is the ring product', () => {
    for (const c of goldenBig('negacyclic.json')) {
      const e = new fhe.PolynomialEngine(c.n, BigInt(c.q), { mode: 'negacyclic' });
      assert.deepStrictEqual(Array.from(e.multiply(U(c.x), U(c.y))), c.product.map(BigInt));
    }
  });
}
Promise.all(asyncTests).then(() => console.log(`${passed} passed (${mode})`)).catch((e) => {
  console.error(e);
  process.exit(1);
});
