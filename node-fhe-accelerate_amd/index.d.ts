// Type declarations of the MI355X backend's JS entry point (lib/index.js).
//
// createEngine() returns the reference's FHEEngine
// (/root/reference/src/api/fhe-engine.ts:33-78) over the types of
// src/api/types.ts:18-166, restated here so a TypeScript caller of the
// reference binds against this package unchanged; the native-level classes
// below (NttContext, DeviceBuffer, PolynomialEngine, GpuFHEEngine) are this
// backend's batched array surface (INTEGRATION.md).  `tsc` is not part of
// this image: tests/test_abi.py checks that every name declared here is
// exported by lib/index.js and every FHEEngine method exists on the engine.

// ---------------------------------------------------------------- handles
// Opaque, frozen handles of device-resident objects (types.ts:18-71).
export interface SecretKey {
  readonly __brand: 'SecretKey';
  readonly handle: bigint;
  readonly keyId: bigint;
}
export interface PublicKey {
  readonly __brand: 'PublicKey';
  readonly handle: bigint;
  readonly keyId: bigint;
}
export interface EvaluationKey {
  readonly __brand: 'EvaluationKey';
  readonly handle: bigint;
  readonly keyId: bigint;
  readonly decompBaseLog: number;
  readonly decompLevel: number;
}
export interface BootstrapKey {
  readonly __brand: 'BootstrapKey';
  readonly handle: bigint;
  readonly keyId: bigint;
  readonly lweDimension: number;
}
export interface Ciphertext {
  readonly __brand: 'Ciphertext';
  readonly handle: bigint;
  readonly keyId: bigint;
  readonly noiseBudget: number;
  readonly isNtt: boolean;
  readonly degree: number;
}
export interface Plaintext {
  readonly __brand: 'Plaintext';
  readonly values: bigint[];
  readonly plaintextModulus: bigint;
  readonly isPacked: boolean;
}

// ---------------------------------------------------------------- parameters (types.ts:77-135)
export type SecurityLevel = 128 | 192 | 256;
export type FHEScheme = 'TFHE' | 'BFV' | 'CKKS';
export type ParameterPreset =
  | 'tfhe-128-fast' | 'tfhe-128-balanced' | 'tfhe-256-secure'
  | 'bfv-128-simd' | 'ckks-128-ml' | 'tfhe-128-voting';
export interface CustomParameters {
  polyDegree: number;
  moduli: bigint[];
  lweDimension?: number;
  lweNoiseStd?: number;
  glweDimension?: number;
  decompBaseLog?: number;
  decompLevel?: number;
  securityLevel: SecurityLevel;
}
export interface ParameterSet {
  scheme: FHEScheme;
  security: SecurityLevel;
  polyDegree: number;
  moduli: bigint[];
  lweDimension: number;
  lweNoiseStd: number;
  glweDimension: number;
  decompBaseLog: number;
  decompLevel: number;
  plaintextModulus: bigint;
  noiseBudget: number;
  maxMultDepth: number;
}

// ---------------------------------------------------------------- errors (types.ts:140-166)
export enum FHEErrorCode {
  NOISE_BUDGET_EXHAUSTED = 'NOISE_BUDGET_EXHAUSTED',
  INVALID_PARAMETERS = 'INVALID_PARAMETERS',
  KEY_MISMATCH = 'KEY_MISMATCH',
  HARDWARE_UNAVAILABLE = 'HARDWARE_UNAVAILABLE',
  SERIALIZATION_ERROR = 'SERIALIZATION_ERROR',
  PROOF_VERIFICATION_FAILED = 'PROOF_VERIFICATION_FAILED',
  THRESHOLD_NOT_MET = 'THRESHOLD_NOT_MET',
  INVALID_BALLOT = 'INVALID_BALLOT',
  DUPLICATE_VOTE = 'DUPLICATE_VOTE',
  NATIVE_ERROR = 'NATIVE_ERROR',
}
export class FHEError extends Error {
  constructor(message: string, code: FHEErrorCode, details?: Record<string, unknown>);
  readonly code: FHEErrorCode;
  readonly details?: Record<string, unknown>;
}

// ---------------------------------------------------------------- hardware (types.ts:171-190)
// The reference's Apple fields, reported false / 0 here, plus the HIP device.
export interface HardwareCapabilities {
  hasSme: boolean;
  hasMetal: boolean;
  hasNeon: boolean;
  hasAmx: boolean;
  hasNeuralEngine: boolean;
  metalGpuCores: number;
  unifiedMemorySize: bigint;
  hasHip?: boolean;
  gpuDevices?: number;
  computeUnits?: number;
  arch?: string;
  name?: string;
}

// ---------------------------------------------------------------- keys, encryption, progress
export type SecretKeyDistribution = 'TERNARY' | 'GAUSSIAN' | 'BINARY' | 'UNIFORM';
export interface KeyGenerationOptions {
  distribution?: SecretKeyDistribution;
  decompBaseLog?: number;
  decompLevel?: number;
}
export interface ThresholdConfig { threshold: number; totalShares: number; }
export interface SecretKeyShare {
  readonly shareId: number;
  readonly handle: bigint;
  readonly commitment: Uint8Array;
  readonly keyId: bigint;
}
export interface ThresholdKeys {
  shares: SecretKeyShare[];
  publicKey: PublicKey;
  threshold: number;
  totalShares: number;
}
export interface PartialDecryption { shareId: number; partialResult: bigint[]; proof?: Uint8Array; }
export interface EncryptionResult { ciphertext: Ciphertext; proof?: Uint8Array; }
export interface DecryptionResult {
  plaintext: Plaintext;
  remainingNoiseBudget: number;
  success: boolean;
  errorMessage?: string;
}
export interface BatchEncryptionOptions { generateProofs?: boolean; useGpu?: boolean; batchSize?: number; }
export interface BatchEncryptionResult {
  ciphertexts: Ciphertext[];
  proofs?: Uint8Array[];
  elapsedMs: number;
  throughputPerSecond: number;
}
export interface ProgressInfo {
  stage: string;
  current: number;
  total: number;
  elapsedMs: number;
  estimatedRemainingMs?: number;
  progressPercent: number;
}
export type ProgressCallback = (progress: ProgressInfo) => void;
export type SerializationFormat = 'binary' | 'json' | 'compressed';
export interface SerializationOptions { format?: SerializationFormat; includeMetadata?: boolean; compress?: boolean; }
export interface SerializedKey {
  data: Uint8Array;
  format: SerializationFormat;
  keyType: 'secret' | 'public' | 'evaluation' | 'bootstrap';
  version: number;
  checksum: Uint8Array;
}
export interface SerializedCiphertext {
  data: Uint8Array;
  format: SerializationFormat;
  keyId: bigint;
  version: number;
  checksum: Uint8Array;
}

// ---------------------------------------------------------------- FHEEngine (fhe-engine.ts:33-78)
export interface FHEEngine {
  generateSecretKey(options?: KeyGenerationOptions): Promise<SecretKey>;
  generatePublicKey(sk: SecretKey): Promise<PublicKey>;
  generateEvalKey(sk: SecretKey, options?: KeyGenerationOptions): Promise<EvaluationKey>;
  generateBootstrapKey(sk: SecretKey): Promise<BootstrapKey>;
  generateThresholdKeys(config: ThresholdConfig): Promise<ThresholdKeys>;
  encrypt(plaintext: Plaintext, pk: PublicKey): Promise<EncryptionResult>;
  encryptValue(value: bigint, pk: PublicKey): Promise<Ciphertext>;
  encryptPacked(values: bigint[], pk: PublicKey): Promise<Ciphertext>;
  decrypt(ciphertext: Ciphertext, sk: SecretKey): Promise<DecryptionResult>;
  decryptValue(ciphertext: Ciphertext, sk: SecretKey): Promise<bigint>;
  decryptPacked(ct: Ciphertext, sk: SecretKey, numValues: number): Promise<bigint[]>;
  batchEncrypt(pts: Plaintext[], pk: PublicKey, opts?: BatchEncryptionOptions): Promise<BatchEncryptionResult>;
  add(ct1: Ciphertext, ct2: Ciphertext): Promise<Ciphertext>;
  addPlain(ct: Ciphertext, pt: Plaintext): Promise<Ciphertext>;
  addScalar(ct: Ciphertext, value: bigint): Promise<Ciphertext>;
  subtract(ct1: Ciphertext, ct2: Ciphertext): Promise<Ciphertext>;
  negate(ct: Ciphertext): Promise<Ciphertext>;
  batchAdd(cts: Ciphertext[], progress?: ProgressCallback): Promise<Ciphertext>;
  multiply(ct1: Ciphertext, ct2: Ciphertext): Promise<Ciphertext>;
  multiplyRelin(ct1: Ciphertext, ct2: Ciphertext, ek: EvaluationKey): Promise<Ciphertext>;
  multiplyPlain(ct: Ciphertext, pt: Plaintext): Promise<Ciphertext>;
  multiplyScalar(ct: Ciphertext, scalar: bigint): Promise<Ciphertext>;
  relinearize(ct: Ciphertext, ek: EvaluationKey): Promise<Ciphertext>;
  square(ct: Ciphertext): Promise<Ciphertext>;
  squareRelin(ct: Ciphertext, ek: EvaluationKey): Promise<Ciphertext>;
  bootstrap(ct: Ciphertext, bk: BootstrapKey): Promise<Ciphertext>;
  programmableBootstrap(ct: Ciphertext, bk: BootstrapKey, lut: bigint[]): Promise<Ciphertext>;
  partialDecrypt(ct: Ciphertext, share: ThresholdKeys['shares'][0]): Promise<PartialDecryption>;
  combinePartialDecryptions(ct: Ciphertext, partials: PartialDecryption[], t: number): Promise<DecryptionResult>;
  getNoiseBudget(ct: Ciphertext, sk: SecretKey): Promise<number>;
  estimateNoiseBudget(ct: Ciphertext): number;
  serializeSecretKey(sk: SecretKey, opts?: SerializationOptions): Promise<SerializedKey>;
  deserializeSecretKey(data: SerializedKey): Promise<SecretKey>;
  serializePublicKey(pk: PublicKey, opts?: SerializationOptions): Promise<SerializedKey>;
  deserializePublicKey(data: SerializedKey): Promise<PublicKey>;
  serializeCiphertext(ct: Ciphertext, opts?: SerializationOptions): Promise<SerializedCiphertext>;
  deserializeCiphertext(data: SerializedCiphertext): Promise<Ciphertext>;
  createPlaintext(value: bigint): Plaintext;
  createPackedPlaintext(values: bigint[]): Plaintext;
  getZeroCiphertext(pk: PublicKey): Promise<Ciphertext>;
  getParams(): ParameterSet;
  getHardwareCapabilities(): HardwareCapabilities;
  getSlotCount(): number;
  dispose(): void;
}

/** Options of this backend (environment defaults FHE_NTT_MODE, FHE_GPU_DEVICES). */
export interface EngineOptions {
  mode?: 'compat' | 'negacyclic';
  device?: number;
  devices?: number[];
}

export declare class FHEEngineImpl implements FHEEngine {
  constructor(params: ParameterSet, options?: EngineOptions);
  generateSecretKey(options?: KeyGenerationOptions): Promise<SecretKey>;
  generatePublicKey(sk: SecretKey): Promise<PublicKey>;
  generateEvalKey(sk: SecretKey, options?: KeyGenerationOptions): Promise<EvaluationKey>;
  generateBootstrapKey(sk: SecretKey): Promise<BootstrapKey>;
  generateThresholdKeys(config: ThresholdConfig): Promise<ThresholdKeys>;
  encrypt(plaintext: Plaintext, pk: PublicKey): Promise<EncryptionResult>;
  encryptValue(value: bigint, pk: PublicKey): Promise<Ciphertext>;
  encryptPacked(values: bigint[], pk: PublicKey): Promise<Ciphertext>;
  decrypt(ciphertext: Ciphertext, sk: SecretKey): Promise<DecryptionResult>;
  decryptValue(ciphertext: Ciphertext, sk: SecretKey): Promise<bigint>;
  decryptPacked(ct: Ciphertext, sk: SecretKey, numValues: number): Promise<bigint[]>;
  batchEncrypt(pts: Plaintext[], pk: PublicKey, opts?: BatchEncryptionOptions): Promise<BatchEncryptionResult>;
  add(ct1: Ciphertext, ct2: Ciphertext): Promise<Ciphertext>;
  addPlain(ct: Ciphertext, pt: Plaintext): Promise<Ciphertext>;
  addScalar(ct: Ciphertext, value: bigint): Promise<Ciphertext>;
  subtract(ct1: Ciphertext, ct2: Ciphertext): Promise<Ciphertext>;
  negate(ct: Ciphertext): Promise<Ciphertext>;
  batchAdd(cts: Ciphertext[], progress?: ProgressCallback): Promise<Ciphertext>;
  multiply(ct1: Ciphertext, ct2: Ciphertext): Promise<Ciphertext>;
  multiplyRelin(ct1: Ciphertext, ct2: Ciphertext, ek: EvaluationKey): Promise<Ciphertext>;
  multiplyPlain(ct: Ciphertext, pt: Plaintext): Promise<Ciphertext>;
  multiplyScalar(ct: Ciphertext, scalar: bigint): Promise<Ciphertext>;
  relinearize(ct: Ciphertext, ek: EvaluationKey): Promise<Ciphertext>;
  square(ct: Ciphertext): Promise<Ciphertext>;
  squareRelin(ct: Ciphertext, ek: EvaluationKey): Promise<Ciphertext>;
  bootstrap(ct: Ciphertext, bk: BootstrapKey): Promise<Ciphertext>;
  programmableBootstrap(ct: Ciphertext, bk: BootstrapKey, lut: bigint[]): Promise<Ciphertext>;
  partialDecrypt(ct: Ciphertext, share: ThresholdKeys['shares'][0]): Promise<PartialDecryption>;
  combinePartialDecryptions(ct: Ciphertext, partials: PartialDecryption[], t: number): Promise<DecryptionResult>;
  getNoiseBudget(ct: Ciphertext, sk: SecretKey): Promise<number>;
  estimateNoiseBudget(ct: Ciphertext): number;
  serializeSecretKey(sk: SecretKey, opts?: SerializationOptions): Promise<SerializedKey>;
  deserializeSecretKey(data: SerializedKey): Promise<SecretKey>;
  serializePublicKey(pk: PublicKey, opts?: SerializationOptions): Promise<SerializedKey>;
  deserializePublicKey(data: SerializedKey): Promise<PublicKey>;
  serializeCiphertext(ct: Ciphertext, opts?: SerializationOptions): Promise<SerializedCiphertext>;
  deserializeCiphertext(data: SerializedCiphertext): Promise<Ciphertext>;
  createPlaintext(value: bigint): Plaintext;
  createPackedPlaintext(values: bigint[]): Plaintext;
  getZeroCiphertext(pk: PublicKey): Promise<Ciphertext>;
  getParams(): ParameterSet;
  getHardwareCapabilities(): HardwareCapabilities;
  getSlotCount(): number;
  dispose(): void;
  /** The device buffer behind a handle (this backend's extension). */
  deviceBuffer(handle: unknown): DeviceBuffer | undefined;
}

/** createEngine (src/index.ts:108): a preset name or custom parameters. */
export function createEngine(params: ParameterPreset | CustomParameters, options?: EngineOptions): Promise<FHEEngine>;
export const createFHEEngine: typeof createEngine;
export function createParameterSet(preset: ParameterPreset): ParameterSet;
export function getAvailablePresets(): ParameterPreset[];
export function calculateDerivedParameters(params: ParameterSet): { noiseBudget: number; maxMultDepth: number };
export const NTT_PRIMES: Record<string, bigint>;

// ---------------------------------------------------------------- native surface
// The reference napi-rs exports (index.d.ts:14-44 of the reference).
export function initialize(): void;
export function detectHardware(): HardwareCapabilities;
export function version(): string;
export declare class ModularArithmetic {
  constructor(modulus: number);
  montgomeryMul(a: number, b: number): number;
  modAdd(a: number, b: number): number;
  modSub(a: number, b: number): number;
  toMontgomery(a: number): number;
  fromMontgomery(a: number): number;
  getModulus(): number;
}

/** u64 coefficient buffers: host arrays (staged through HBM per call) or
 * DeviceBuffers of the same context (device-resident). */
export type Words = BigUint64Array | DeviceBuffer;

export interface NttContextInfo {
  degree: number;
  modulus: bigint;
  primitiveRoot: bigint;
  mode: number;
  devices: number;
  [key: string]: unknown;
}

/** One libfhe_gpu context (fhe_ctx_create / fhe_ctx_create_multi).  Every
 * compute method X has a promise form XAsync (napi_async_work). */
export declare class NttContext {
  constructor(degree: number, modulus: bigint | number, mode?: number, device?: number | number[]);
  info(): NttContextInfo;
  synchronize(): void;
  /** Ciphertexts of two-CU blind rotations recomputed by the one-CU repair pass
   * (a partner workgroup was not co-resident; results are exact either way). */
  brRepairCount(): number;
  forward(a: Words, out?: Words): Words;
  inverse(a: Words, out?: Words): Words;
  polymul(a: Words, b: Words, out: Words): Words;
  pointwise(a: Words, b: Words, out: Words): Words;
  forwardMul(a: Words, w: Words, out: Words): Words;
  add(a: Words, b: Words, out: Words): Words;
  sub(a: Words, b: Words, out: Words): Words;
  negate(a: Words, out: Words): Words;
  mulScalar(a: Words, s: bigint, out: Words): Words;
  ctMultiply(ct1: Words, ct2: Words, out: Words, isNtt?: number): Words;
  relinearize(ct3: Words, rlk: Words, baseLog: number, out: Words): Words;
  externalProduct(glwe: Words, ggsw: Words, baseLog: number, level: number, out: Words): Words;
  blindRotate(acc: Words, lweA: Words, lweB: Words, bsk: Words, baseLog: number, level: number): Words;
  forwardAsync(a: Words, out?: Words): Promise<Words>;
  inverseAsync(a: Words, out?: Words): Promise<Words>;
  polymulAsync(a: Words, b: Words, out: Words): Promise<Words>;
  ctMultiplyAsync(ct1: Words, ct2: Words, out: Words, isNtt?: number): Promise<Words>;
  relinearizeAsync(ct3: Words, rlk: Words, baseLog: number, out: Words): Promise<Words>;
  [method: string]: unknown;
}

/** Device memory of one NttContext (refcounted; views share it). */
export declare class DeviceBuffer {
  constructor(ctx: NttContext, words: number);
  constructor(parent: DeviceBuffer, offsetWords: number, words: number);
  readonly words: number;
  readonly handle: bigint;
  upload(src: BigUint64Array | BigInt64Array, offsetWords?: number): this;
  download(dst?: BigUint64Array, offsetWords?: number, words?: number): BigUint64Array;
  copyFrom(src: DeviceBuffer, dstOffset?: number, srcOffset?: number, words?: number): this;
  view(offsetWords: number, words: number): DeviceBuffer;
  free(): void;
}

export function modmulBatch(q: bigint, a: BigUint64Array, b: BigUint64Array, out: BigUint64Array): BigUint64Array;
export function mlMontgomeryMulBatch(q: BigUint64Array, a: BigUint64Array, b: BigUint64Array,
                                     out: BigUint64Array): BigUint64Array;

/** Batched polynomial arithmetic over Z_q[X] (array level). */
export declare class PolynomialEngine {
  constructor(degree: number, modulus: bigint | number, opts?: EngineOptions);
  readonly degree: number;
  readonly modulus: bigint;
  alloc(batch?: number): BigUint64Array;
  toNtt(a: Words, out?: Words): Words;
  fromNtt(a: Words, out?: Words): Words;
  multiply(a: Words, b: Words, out?: Words): Words;
  pointwiseMultiply(a: Words, b: Words, out?: Words): Words;
  add(a: Words, b: Words, out?: Words): Words;
  subtract(a: Words, b: Words, out?: Words): Words;
  negate(a: Words, out?: Words): Words;
  multiplyScalar(a: Words, s: bigint | number, out?: Words): Words;
  forwardMultiply(a: Words, w: Words, out?: Words): Words;
  externalProduct(glwe: Words, ggsw: Words, baseLog: number, level: number, out?: Words): Words;
  ctMultiply(ct1: Words, ct2: Words, opts?: { isNtt?: boolean }, out?: Words): Words;
  relinearize(ct3: Words, rlk: Words, baseLog?: number, out?: Words): Words;
  multiplyRelin(ct1: Words, ct2: Words, rlk: Words, baseLog?: number): Words;
  blindRotate(acc: Words, lweA: Words, lweB: Words, bsk: Words, baseLog: number, level: number): Words;
  brRepairCount(): number;
  info(): NttContextInfo;
}

/** The FHEEngine operations at array level (ciphertexts as BigUint64Array). */
export declare class GpuFHEEngine {
  constructor(params: ParameterPreset | Partial<ParameterSet> & { polyDegree: number; moduli: bigint[] },
              opts?: EngineOptions);
  readonly n: number;
  readonly q: bigint;
  readonly t: bigint;
  getSlotCount(): number;
  [method: string]: unknown;
}

export const PRESETS: Record<ParameterPreset, Partial<ParameterSet> & { polyDegree: number; moduli: bigint[] }>;
export const sampling: {
  uniformMod(q: bigint, count: number): BigUint64Array;
  ternary(q: bigint, count: number): BigUint64Array;
  gaussian(q: bigint, std: number, count: number): BigUint64Array;
};
