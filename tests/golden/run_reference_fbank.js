// Runs the reference's own executable fbank -- computeFbank() of
// /root/reference/offline_pwa/static/js/pure-ort-asr-worker.js:470-519 (window :359-367,
// Hz-domain mel triangles :369-397, radix-2 FFT :399-458, reflection :460-468) -- under node,
// on raw float32 inputs, and writes its raw float32 outputs.  Test infrastructure only, run by
// tests/golden/make_golden_fbank_js.py in the build container (the reference is not on the
// GPU box).
//
// The worker file is untrusted input, so it is NOT evaluated as a whole.  This script reads it
// as text and cuts out exactly the pieces the fbank needs:
//   * the numeric constants SAMPLE_RATE .. LOG_FLOOR (:3-11), each checked to be one numeric
//     literal and re-emitted from the parsed number;
//   * the function declarations hzToMel, melToHz, getAsrWindow, getAsrMelBank, getFftTables,
//     fftInPlace, reflectIndex, computeFbank (brace-matched), each checked against a deny list
//     of identifiers that could reach outside the computation (require, process, import,
//     eval, Function, constructor, globalThis, this, self, postMessage, fetch, ...);
// and evaluates only that text in a vm context made from a null-prototype object: no host
// object (console, Buffer, the sandbox's prototype) is passed in, so the code sees the
// context's own built-ins and nothing else.  Inputs go in as context-realm Float32Arrays
// filled element by element; outputs come back as plain numbers.  The caller runs this file
// in a child process with an empty environment in a scratch directory.
//
// One change to the extracted text: this container's node (v12) predates optional chaining,
// so `samples?.length` in computeFbank is rewritten to `(samples == null ? undefined :
// samples.length)` -- a syntax lowering that leaves every arithmetic operation as written.
//
// usage: node run_reference_fbank.js <worker.js> <in.f32> <lengths comma-separated> <out.f32>
"use strict";
const fs = require("fs");
const vm = require("vm");

const [workerPath, inPath, lensArg, outPath] = process.argv.slice(2);
const text = fs.readFileSync(workerPath, "utf8");

const CONSTS = ["SAMPLE_RATE", "FRAME_LENGTH", "FRAME_SHIFT", "N_FFT", "NUM_MEL_BINS", "LOW_FREQ",
                "HIGH_FREQ", "PREEMPHASIS", "LOG_FLOOR"];
const FUNCS = ["hzToMel", "melToHz", "getAsrWindow", "getAsrMelBank", "getFftTables",
               "fftInPlace", "reflectIndex", "computeFbank"];
const DENY = ["require", "process", "import", "eval", "Function", "constructor", "prototype",
              "__proto__", "globalThis", "this", "self", "postMessage", "fetch", "global",
              "Reflect", "Proxy", "setTimeout", "setInterval", "WebAssembly", "Atomics",
              "SharedArrayBuffer", "ort", "importScripts", "`"];

let code = "";
for (const name of CONSTS) {
  const m = text.match(new RegExp("^const " + name + " = ([0-9][0-9.eE+-]*);$", "m"));
  if (!m) throw new Error("constant " + name + " not found as a numeric literal");
  const v = Number(m[1]);
  if (!Number.isFinite(v)) throw new Error("constant " + name + " is not a finite number");
  code += "const " + name + " = " + String(v) + ";\n";
}
code += "let fftTables = null;\nlet asrWindow = null;\nlet asrMelBank = null;\n";

function extractFunction(name) {
  const head = "\nfunction " + name + "(";
  const at = text.indexOf(head);
  if (at < 0 || text.indexOf(head, at + 1) >= 0) throw new Error("function " + name + ": not unique");
  const open = text.indexOf("{", at);
  let depth = 0;
  for (let i = open; i < text.length; i += 1) {
    const c = text[i];
    if (c === '"' || c === "'" || c === "`" || (c === "/" && (text[i + 1] === "/" || text[i + 1] === "*")))
      throw new Error("function " + name + ": strings / comments / templates are not expected");
    if (c === "{") depth += 1;
    else if (c === "}") {
      depth -= 1;
      if (depth === 0) return text.slice(at + 1, i + 1);
    }
  }
  throw new Error("function " + name + ": unbalanced braces");
}

for (const name of FUNCS) {
  let body = extractFunction(name);
  body = body.replace(/\bsamples\?\.length\b/g, "(samples == null ? undefined : samples.length)");
  if (body.includes("?.")) throw new Error(name + ": optional chaining left after lowering");
  for (const bad of DENY) {
    const re = bad === "`" ? /`/ : new RegExp("\\b" + bad.replace(/[$]/g, "\\$") + "\\b");
    if (re.test(body)) throw new Error(name + ": denied identifier " + bad);
  }
  code += body + "\n";
}

const sandbox = Object.create(null);
const ctx = vm.createContext(sandbox);
vm.runInContext(code, ctx, { filename: "fbank-extract.js", timeout: 60000 });
// context-realm helpers, called with numbers and context-realm arrays only (no host
// function or object ever reaches the extracted code)
const makeInput = vm.runInContext("(function (n) { return new Float32Array(n); })", ctx);
const run = vm.runInContext(
  "(function (x) { const r = computeFbank(x); const out = new Float32Array(r.data.length);" +
  " for (let i = 0; i < out.length; i += 1) out[i] = r.data[i]; return [+r.frames, out]; })", ctx);

const raw = fs.readFileSync(inPath);
const all = new Float32Array(raw.buffer, raw.byteOffset, raw.byteLength / 4);
const lens = lensArg.split(",").map((x) => parseInt(x, 10));
const outs = [];
let off = 0;
for (const n of lens) {
  const x = makeInput(n);
  for (let i = 0; i < n; i += 1) x[i] = all[off + i];
  off += n;
  const res = run(x);
  const frames = Number(res[0]);
  const data = res[1];
  if (!(frames * 80 === data.length)) throw new Error("bad output size");
  const f = new Float32Array(data.length);
  for (let i = 0; i < f.length; i += 1) f[i] = Number(data[i]);
  outs.push(Buffer.from(f.buffer));
}
fs.writeFileSync(outPath, Buffer.concat(outs));
process.stdout.write(JSON.stringify({ inputs: lens.length, samples: off, functions: FUNCS.length }) + "\n");
