"""Host runtime around the engine: service loop, sinks, queues, supervisor, notifier, JMX."""
