-- llm_mcp_amd Postgres schema: one idempotent script applied at startup by
-- PostgresStore.migrate() (the reference ships 01_core.sql as initdb plus four
-- hand-applied migrations that the code silently depends on; SURVEY §2.2).
-- Table and column names follow the reference contract
-- (db/init/01_core.sql, db/migrations/02..05) so existing dashboards/queries
-- keep working; additions are marked "lmx:".

CREATE EXTENSION IF NOT EXISTS pgcrypto;

CREATE TABLE IF NOT EXISTS devices (
  id          TEXT PRIMARY KEY,
  name        TEXT,
  platform    TEXT,
  arch        TEXT,
  host        TEXT,
  tags        JSONB NOT NULL DEFAULT '{}',
  status      TEXT NOT NULL DEFAULT 'unknown',
  last_seen   TIMESTAMPTZ,
  created_at  TIMESTAMPTZ NOT NULL DEFAULT now(),
  updated_at  TIMESTAMPTZ NOT NULL DEFAULT now()
);

CREATE TABLE IF NOT EXISTS device_metrics (
  id            UUID PRIMARY KEY DEFAULT gen_random_uuid(),
  device_id     TEXT NOT NULL REFERENCES devices(id) ON DELETE CASCADE,
  ts            TIMESTAMPTZ NOT NULL DEFAULT now(),
  cpu_pct       NUMERIC,
  mem_used_mb   INT,
  mem_total_mb  INT,
  gpu_name      TEXT,
  vram_used_mb  INT,
  vram_total_mb INT,
  tps           NUMERIC,
  latency_ms    INT,
  notes         JSONB
);
CREATE INDEX IF NOT EXISTS device_metrics_dev_ts ON device_metrics (device_id, ts DESC);

CREATE TABLE IF NOT EXISTS models (
  id          TEXT PRIMARY KEY,
  provider    TEXT NOT NULL DEFAULT 'local',
  family      TEXT,
  kind        TEXT NOT NULL DEFAULT 'chat',
  params_b    NUMERIC,
  context_k   INT,
  size_gb     NUMERIC,
  quant       TEXT,
  status      TEXT NOT NULL DEFAULT 'active',
  tier        TEXT,
  thinking    BOOLEAN NOT NULL DEFAULT FALSE,
  meta        JSONB,
  updated_at  TIMESTAMPTZ NOT NULL DEFAULT now()
);

CREATE TABLE IF NOT EXISTS model_pricing (
  model_id     TEXT PRIMARY KEY,
  price_in_1m  NUMERIC,
  price_out_1m NUMERIC,
  currency     TEXT NOT NULL DEFAULT 'USD',
  updated_at   TIMESTAMPTZ NOT NULL DEFAULT now()
);

CREATE TABLE IF NOT EXISTS device_models (
  device_id     TEXT NOT NULL REFERENCES devices(id) ON DELETE CASCADE,
  model_id      TEXT NOT NULL,
  available     BOOLEAN NOT NULL DEFAULT TRUE,
  max_context_k INT,
  meta          JSONB,
  updated_at    TIMESTAMPTZ NOT NULL DEFAULT now(),
  PRIMARY KEY (device_id, model_id)
);

CREATE TABLE IF NOT EXISTS benchmarks (
  id          UUID PRIMARY KEY DEFAULT gen_random_uuid(),
  device_id   TEXT NOT NULL,
  model_id    TEXT NOT NULL,
  task_type   TEXT NOT NULL,
  tokens_in   INT,
  tokens_out  INT,
  latency_ms  INT,
  tps         NUMERIC,
  meta        JSONB,
  ok          BOOLEAN NOT NULL DEFAULT TRUE,
  created_at  TIMESTAMPTZ NOT NULL DEFAULT now()
);
CREATE INDEX IF NOT EXISTS benchmarks_model_task ON benchmarks (model_id, task_type, created_at DESC);

CREATE TABLE IF NOT EXISTS jobs (
  id            UUID PRIMARY KEY DEFAULT gen_random_uuid(),
  kind          TEXT NOT NULL,
  payload       JSONB NOT NULL DEFAULT '{}',
  priority      INT NOT NULL DEFAULT 0,
  status        TEXT NOT NULL DEFAULT 'queued',
  source        TEXT,
  attempts      INT NOT NULL DEFAULT 0,
  max_attempts  INT NOT NULL DEFAULT 3,
  lease_until   TIMESTAMPTZ,
  deadline_at   TIMESTAMPTZ,
  result        JSONB,
  error         TEXT,
  queued_at     TIMESTAMPTZ NOT NULL DEFAULT now(),
  updated_at    TIMESTAMPTZ NOT NULL DEFAULT now()
);
-- lmx: placement + lease ownership (a stale worker cannot complete a job it lost)
ALTER TABLE jobs ADD COLUMN IF NOT EXISTS device_id   TEXT;
ALTER TABLE jobs ADD COLUMN IF NOT EXISTS worker_id   TEXT;
ALTER TABLE jobs ADD COLUMN IF NOT EXISTS lease_token UUID;
-- lmx: last progress report of the lease owner (tokens so far), streamed by SSE
ALTER TABLE jobs ADD COLUMN IF NOT EXISTS progress    JSONB;
CREATE INDEX IF NOT EXISTS jobs_claim ON jobs (status, priority DESC, queued_at);
CREATE INDEX IF NOT EXISTS jobs_lease ON jobs (lease_until);
CREATE INDEX IF NOT EXISTS jobs_device_running ON jobs (device_id) WHERE status = 'running';
CREATE INDEX IF NOT EXISTS jobs_updated ON jobs (updated_at DESC, status);

CREATE TABLE IF NOT EXISTS job_attempts (
  id          UUID PRIMARY KEY DEFAULT gen_random_uuid(),
  job_id      UUID NOT NULL REFERENCES jobs(id) ON DELETE CASCADE,
  worker_id   TEXT,
  started_at  TIMESTAMPTZ NOT NULL DEFAULT now(),
  finished_at TIMESTAMPTZ,
  status      TEXT NOT NULL DEFAULT 'running',
  error       TEXT,
  metrics     JSONB
);
CREATE INDEX IF NOT EXISTS job_attempts_job ON job_attempts (job_id, started_at);

CREATE TABLE IF NOT EXISTS device_limits (
  device_id       TEXT PRIMARY KEY,
  ram_gb          NUMERIC,
  vram_gb         NUMERIC,
  max_params_b    NUMERIC,
  max_size_gb     NUMERIC,
  max_context_k   INT,
  allow_models    JSONB,
  deny_models     JSONB,
  max_concurrency INT,
  spec            JSONB,          -- lmx: full limit spec as applied
  updated_at      TIMESTAMPTZ NOT NULL DEFAULT now()
);

CREATE TABLE IF NOT EXISTS llm_costs (
  id          UUID PRIMARY KEY DEFAULT gen_random_uuid(),
  job_id      UUID,
  model_id    TEXT NOT NULL,
  provider    TEXT NOT NULL,
  tokens_in   INT NOT NULL DEFAULT 0,
  tokens_out  INT NOT NULL DEFAULT 0,
  cost_usd    NUMERIC NOT NULL DEFAULT 0,
  currency    TEXT NOT NULL DEFAULT 'USD',
  created_at  TIMESTAMPTZ NOT NULL DEFAULT now()
);
CREATE INDEX IF NOT EXISTS llm_costs_created ON llm_costs (created_at DESC);

CREATE OR REPLACE VIEW v_cost_stats AS
  SELECT date_trunc('day', created_at) AS day, provider, model_id,
         COUNT(*) AS requests, SUM(tokens_in) AS tokens_in, SUM(tokens_out) AS tokens_out,
         SUM(cost_usd) AS cost_usd
  FROM llm_costs GROUP BY 1, 2, 3;

CREATE OR REPLACE FUNCTION calculate_job_cost(p_model_id TEXT, p_tokens_in INT, p_tokens_out INT)
RETURNS NUMERIC AS $$
  SELECT COALESCE((SELECT COALESCE(price_in_1m, 0) * p_tokens_in / 1000000.0
                        + COALESCE(price_out_1m, 0) * p_tokens_out / 1000000.0
                   FROM model_pricing WHERE model_id = p_model_id), 0);
$$ LANGUAGE sql STABLE;

CREATE OR REPLACE FUNCTION notify_job_status_change() RETURNS trigger AS $$
BEGIN
  IF TG_OP = 'INSERT' OR NEW.status IS DISTINCT FROM OLD.status
     OR NEW.progress IS DISTINCT FROM OLD.progress THEN
    PERFORM pg_notify('job_update', NEW.id::text);
  END IF;
  RETURN NEW;
END;
$$ LANGUAGE plpgsql;

DROP TRIGGER IF EXISTS trg_job_status_notify ON jobs;
CREATE TRIGGER trg_job_status_notify AFTER INSERT OR UPDATE ON jobs
  FOR EACH ROW EXECUTE FUNCTION notify_job_status_change();

CREATE TABLE IF NOT EXISTS model_rankings (
  model_id           TEXT PRIMARY KEY,
  provider           TEXT NOT NULL DEFAULT 'openrouter',
  display_name       TEXT,
  category_scores    JSONB DEFAULT '{}',
  context_k          INT,
  price_in_1m        NUMERIC,
  price_out_1m       NUMERIC,
  modalities         JSONB DEFAULT '["text"]',
  supports_streaming BOOLEAN DEFAULT TRUE,
  supports_tools     BOOLEAN DEFAULT FALSE,
  supports_vision    BOOLEAN DEFAULT FALSE,
  is_local           BOOLEAN DEFAULT FALSE,
  updated_at         TIMESTAMPTZ DEFAULT now()
);

CREATE TABLE IF NOT EXISTS model_stats (
  model_id          TEXT PRIMARY KEY,
  total_requests    INT DEFAULT 0,
  total_tokens_in   BIGINT DEFAULT 0,
  total_tokens_out  BIGINT DEFAULT 0,
  total_cost_usd    NUMERIC DEFAULT 0,
  avg_duration_ms   NUMERIC DEFAULT 0,
  error_count       INT DEFAULT 0,
  last_used_at      TIMESTAMPTZ,
  feedback_positive INT DEFAULT 0,
  feedback_negative INT DEFAULT 0,
  success_rate NUMERIC GENERATED ALWAYS AS (
    CASE WHEN total_requests > 0
         THEN round((total_requests - error_count)::numeric * 100 / total_requests, 2)
         ELSE 0 END) STORED,
  avg_cost_per_request NUMERIC GENERATED ALWAYS AS (
    CASE WHEN total_requests > 0 THEN total_cost_usd / total_requests ELSE 0 END) STORED,
  updated_at        TIMESTAMPTZ DEFAULT now()
);

-- 7-day per-device job statistics (reference: 04_smart_routing.sql v_device_stats)
CREATE OR REPLACE VIEW v_device_stats AS
  SELECT j.device_id,
         COUNT(*) AS total_jobs_7d,
         COUNT(*) FILTER (WHERE j.status = 'done') AS done_jobs_7d,
         AVG((a.metrics->>'ms')::numeric) FILTER (WHERE a.status = 'done') AS avg_latency_ms
  FROM jobs j LEFT JOIN job_attempts a ON a.job_id = j.id AND a.status = 'done'
  WHERE j.updated_at > now() - interval '7 days' AND j.status IN ('done', 'error')
  GROUP BY j.device_id;
