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
      }
      assert.deepStrictEqual(Array.from(got), c.out.map(BigInt), `${c.op} n=${c.n}`);
    }
  });
  test('createEngine: ciphertext multiply / relinearize vs golden (async FHEEngine surface)', () => {
    const pending = [];
    for (const c of goldenBig('cipher.json')) {
      if (c.op === 'blind_rotate') continue;
      const custom = { polyDegree: c.n, moduli: [BigInt(c.q)], decompBaseLog: c.base_log || 4 };
      pending.push(fhe.createEngine(custom).then(async (eng) => {
        const got = c.op === 'ct_multiply' ? await eng.multiply(U(c.ct1), U(c.ct2))
          : await eng.relinearize(U(c.ct3), U(c.rlk), c.base_log);
        assert.deepStrictEqual(Array.from(got), c.out.map(BigInt), `${c.op} n=${c.n}`);
      }));
    }
    asyncTests.push(Promise.all(pending));
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
